#!/bin/bash
# Config 4 FUSED: narrow groups in chunk-major chunks of one group per XCD, so a launch's voltage
# rows (16 replicas x 200 KB per XCD at W = 16) stay in the XCD's 4 MB L2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/cfg4l2; mkdir -p $OUT
run() { timeout -k 10 300 "$@" >> $OUT/bench.jsonl 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
        tail -1 $OUT/bench.jsonl | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['algorithm'], d['chunk'], d['schedule'], d['env'], round(d['ms_per_step'],4), round(d['algorithmic_GBps']))"; }
B="python scripts/bench_configs.py --configs config4 --steps 20 --warmup 3 --no-cpu"
run $B
ODESAT_GROUP_WIDTH=16 run $B
ODESAT_GROUP_WIDTH=16 run $B --chunk 128 --schedule 2
ODESAT_GROUP_WIDTH=16 run $B --chunk 256 --schedule 2
ODESAT_GROUP_WIDTH=8 run $B --chunk 64 --schedule 2
ODESAT_GROUP_WIDTH=8 run $B --chunk 128 --schedule 2
ODESAT_GROUP_WIDTH=32 run $B --chunk 256 --schedule 2
