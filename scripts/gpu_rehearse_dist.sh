#!/bin/bash
# Rehearsal of the driver's SCALE shapes on one GPU: every leg at world 2 over gloo (two ranks sharing
# the device) and at world 1 with a process group over RCCL (ODESAT_BENCH_DIST=1).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ODESAT_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu \
    > gpurun_out/bench_w2_all.log 2>&1 || { echo "w2 rc=$?"; tail -20 gpurun_out/bench_w2_all.log; exit 1; }
grep '^{' gpurun_out/bench_w2_all.log > gpurun_out/bench_w2_all.json; echo "w2 ok"
ODESAT_BENCH_DIST=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
    --master-addr 127.0.0.1 --master-port 29534 bench.py --steps 20 --warmup 5 --no-cpu \
    > gpurun_out/bench_rccl_w1.log 2>&1 || { echo "rccl w1 rc=$?"; tail -20 gpurun_out/bench_rccl_w1.log; exit 1; }
grep '^{' gpurun_out/bench_rccl_w1.log > gpurun_out/bench_rccl_w1.json; echo "rccl w1 ok"
