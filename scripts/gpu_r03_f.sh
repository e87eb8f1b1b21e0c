# round 3 measurement: the driver-shaped bench line (every leg, PMC fits from profiles/), the
# 200-step headline, the rocprofv3 kernel stats of the headline alone (warmup launch as long as the
# timed one), and a world-2 rehearsal of the multi-GPU legs (two gloo ranks sharing the GPU).
set -u
mkdir -p gpurun_out
SKIPALL=f64,adaptive,inter,config4,config5,extra,ab
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_f.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_f.log; exit 1; }
grep '^{' gpurun_out/bench_f.log > gpurun_out/bench_f.json; echo "bench20 ok"
timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --skip $SKIPALL --no-cpu > gpurun_out/bench_f200.log 2>&1 || { echo "bench200 rc=$?"; exit 1; }
grep '^{' gpurun_out/bench_f200.log > gpurun_out/bench_f200.json; echo "bench200 ok"
export TMPDIR=/tmp
ROOT=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/rocprof_f" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 20 --skip $SKIPALL --no-cpu > "$ROOT/gpurun_out/rocprof_f.log" 2>&1 || { echo "rocprof rc=$?"; exit 1; }
cd "$ROOT"
echo "rocprof ok"
ODESAT_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --only config4,config5 --no-cpu \
    > gpurun_out/bench_w2.log 2>&1 || { echo "w2 rc=$?"; tail -20 gpurun_out/bench_w2.log; exit 1; }
grep '^{' gpurun_out/bench_w2.log > gpurun_out/bench_w2.json; echo "w2 ok"
