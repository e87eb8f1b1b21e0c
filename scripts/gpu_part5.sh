#!/bin/bash
# Config 5 (n = 1M, m = 4.2M) at world 1: the partitioned step's variants, then the kernel stats of the
# default one.  Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/part5; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_partition.py tests/test_gpu_configs.py -k "partition or config5" -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for v in ${VARIANTS:-"variables minvar 0 region 1 0 16 1" "variables minvar 0 region 1 0 16 0" "clauses minvar 0 region 1 0 16 1"}; do
    set -- $v
    ODESAT_PART_TERMS=$4 ODESAT_PART_K3=$5 ODESAT_PART_XCD=$6 ODESAT_PART_REGIONS=$7 ODESAT_PART_PACK=${8:-1} timeout -k 10 300 python scripts/bench_partition.py --mode $1 --order $2 --graph $3 --steps 200 --warmup 20 \
        >> $OUT/bench.jsonl 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    tail -1 $OUT/bench.jsonl | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['config']['mode'], d['config']['order'], d['config']['terms'], 'k3=$5 xcd=$6 rg=$7 pack=${8:-1}', d['config']['graph_steps'], round(d['ms_per_step'],4))"
done
export TMPDIR=/tmp
ROOT=$(pwd)
cd /tmp
ODESAT_PART_TERMS=${RT:-region} ODESAT_PART_XCD=${RX:-0} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/rocprof -o run --output-format csv -- \
    python3 $ROOT/scripts/bench_partition.py --mode variables --steps 200 --warmup 20 > $ROOT/$OUT/rocprof.log 2>&1 || exit 1
cd $ROOT
find $OUT/rocprof -name '*kernel_stats.csv' -exec head -8 {} \;
