#!/bin/bash
# bench.py --gpus 8 rehearsed on ONE GPU (VERDICT r4 "Next #1"): 8 ranks over gloo sharing the box's
# device (ODESAT_DIST_BACKEND=gloo; dist_setup maps the ranks onto the visible GPU round-robin), every
# leg, with the in-run digests: config 4's replicas re-integrated by rank 0 for every rank, config 5's
# three partitions at world 8 against a world-1 VARIABLES run.  Timing is not the point (8 ranks share
# one device); the JSON line is kept as profiles/<tag>_bench_world8_gloo_one_gpu.json.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-w8}
mkdir -p "$OUT"
export ODESAT_DIST_BACKEND=gloo
timeout -k 20 1100 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port ${PORT:-29531} bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu --steady-calls 0 \
    > "$OUT/bench_w8.log" 2>&1 || { echo "world-8 bench rc=$?"; tail -20 "$OUT/bench_w8.log"; exit 1; }
grep '^{' "$OUT/bench_w8.log" | tail -1 > "$OUT/bench_w8.json"
python3 - "$OUT/bench_w8.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c4, c5 = d.get("inter_config4", {}), d.get("partition_config5", {})
print("ranks", d["ranks"], "value", round(d["value"]), "config4 digest", (c4.get("digest") or {}).get("match"),
      "config5 digest", c5.get("digest"), "errors", {k: v["error"] for k, v in d.items() if isinstance(v, dict) and "error" in v})
PY
