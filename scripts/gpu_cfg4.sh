#!/bin/bash
# Config 4 (n = 50k, m = 210k, B = 1024, fixed dt): FUSED variants and the default's PMC traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/cfg4; mkdir -p $OUT
run() { timeout -k 10 300 "$@" >> $OUT/bench.jsonl 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
        tail -1 $OUT/bench.jsonl | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['algorithm'], d['chunk'], d['schedule'], d['env'], round(d['ms_per_step'],4), round(d['algorithmic_GBps']))"; }
run python scripts/bench_configs.py --configs config4 --steps 50 --warmup 5 --no-cpu
ODESAT_RB=8 run python scripts/bench_configs.py --configs config4 --steps 50 --warmup 5 --no-cpu
run python scripts/bench_configs.py --configs config4 --steps 50 --warmup 5 --no-cpu --chunk 64 --schedule 2
run python scripts/bench_configs.py --configs config4 --steps 50 --warmup 5 --no-cpu --chunk 128 --schedule 2
run python scripts/bench_configs.py --configs config4 --steps 50 --warmup 5 --no-cpu --chunk 256 --schedule 2
ODESAT_GROUP_WIDTH=32 run python scripts/bench_configs.py --configs config4 --steps 50 --warmup 5 --no-cpu
run python scripts/bench_configs.py --configs config4 --steps 50 --warmup 5 --no-cpu --alg twopass
CONFIG=config4 STEPS=5 ALG=0 TAG=r02_cfg4 PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum|SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
    bash scripts/pmc.sh > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
echo pmc ok
