#!/bin/bash
# k_wave waves-per-replica sweep on config 3 (adaptive and fixed dt) at several batches.  Each GPU
# step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/wave_sweep; mkdir -p $OUT
for cfg in config3 config3f; do
  for B in 256 1024 4096; do
    for team in auto 1 2 4; do
      if [ $team = auto ]; then unset ODESAT_WAVE_TEAM; else export ODESAT_WAVE_TEAM=$team; fi
      timeout -k 10 300 python scripts/bench_configs.py --configs $cfg --batch $B --no-cpu --steps 200 > $OUT/r.jsonl 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
      python3 - $OUT/r.jsonl "$cfg B=$B team=$team" <<'PY' | tee -a $OUT/summary.txt
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[2], round(d["replica_steps_per_s"] / 1e6, 2), "M", round(d["ms_per_step"], 4), "ms")
PY
    done
  done
done
