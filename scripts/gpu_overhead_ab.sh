#!/bin/bash
# Round 4: what a headline call costs beside its kernel: the first call after the warm-up against the
# rest, with the warm-up call itself profiled (PROFILE_WARMUP=1) or not.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-overhead}
mkdir -p "$OUT"
for pw in 0 1 0 1; do
  PROFILE_WARMUP=$pw CALLS=6 timeout -k 10 120 python -u scripts/probe_call_overhead.py > "$OUT/ov_pw$pw.json" 2>/dev/null || exit 1
  echo "profile_warmup=$pw $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(round(d["kernel_us_median"],1), d["overhead_us"])' "$OUT/ov_pw$pw.json")"
done
