#!/bin/bash
# GPU: the CLI tests, the N=2 bench path rehearsed on one GPU (gloo), and the partitioned instance
# at world 2 on one GPU (gloo, both partitions).  Each GPU step has its own limit; failures end it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/cli
mkdir -p $OUT
run() {  # run NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -4 "$OUT/$name.log"
    return $rc
}
export ODESAT_DIST_BACKEND=gloo
run pytest_cli 300 python -u -m pytest tests/test_cli.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
run bench_n2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 200 --warmup 50 --no-cpu --no-ab || exit $?
run part_w2_var 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 scripts/bench_partition.py --gpus 2 --config config5 --mode variables --steps 20 --warmup 5 || exit $?
run part_w2_cla 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 scripts/bench_partition.py --gpus 2 --config config5 --mode clauses --steps 20 --warmup 5 || exit $?
