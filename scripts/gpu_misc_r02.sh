#!/bin/bash
# Round-2 GPU session: PMC of the partitioned kernels (config 5), the multi-rank bench path rehearsed
# over gloo with two ranks on the box's GPU, and the k_onchip wave-priority experiment.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/misc; mkdir -p $OUT
PROG=scripts/bench_partition.py PROG_ARGS="--steps 20 --warmup 0 --graph 0" TAG=r02_part5 \
    PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE|TCC_HIT_sum TCC_MISS_sum" \
    bash scripts/pmc.sh > $OUT/pmc_part5.log 2>&1 || { tail -20 $OUT/pmc_part5.log; exit 1; }
echo "pmc ok"
ODESAT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-ab \
    > $OUT/bench_rehearsal_w2.log 2>&1 || { tail -30 $OUT/bench_rehearsal_w2.log; exit 1; }
grep '^{' $OUT/bench_rehearsal_w2.log | cut -c1-400
for pr in 0 1 2; do
    ODESAT_ONCHIP_PRIO=$pr timeout -k 10 300 python bench.py --steps 200 --warmup 50 --no-cpu --no-ab --no-inter \
        --extra-batch 0 > $OUT/bench_prio$pr.log 2>&1 || { tail -20 $OUT/bench_prio$pr.log; exit 1; }
    grep '^{' $OUT/bench_prio$pr.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('prio', $pr, d['value'], d['ms_per_step'])"
done
