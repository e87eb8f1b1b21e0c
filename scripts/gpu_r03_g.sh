# round 3: the RCCL paths of the multi-GPU legs rehearsed on one GPU (a world-1 nccl process group:
# TorchComm over RCCL, RCCL calls captured in the config-5 HIP graphs), the criterion benches, smoke.
set -u
mkdir -p gpurun_out
ODESAT_BENCH_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
    --master-addr 127.0.0.1 --master-port 29541 bench.py --steps 20 --warmup 5 --only config4,config5 --no-cpu \
    > gpurun_out/bench_rccl1.log 2>&1 || { echo "rccl1 rc=$?"; tail -20 gpurun_out/bench_rccl1.log; exit 1; }
grep '^{' gpurun_out/bench_rccl1.log > gpurun_out/bench_rccl1.json; echo "rccl1 ok"
python -c "import json; d=json.load(open('gpurun_out/bench_rccl1.json')); c=d['partition_config5']; print({k: c[k].get('value', c[k]) if isinstance(c[k], dict) else c[k] for k in ('clauses','clauses_rs','variables','backend')}); print(c.get('digest')); print(d['inter_config4'].get('digest'), d['inter_config4'].get('value'))"
timeout -k 10 300 python -u scripts/bench_criterion.py > gpurun_out/crit3.jsonl 2>&1 || { echo "crit rc=$?"; exit 1; }
grep '^{' gpurun_out/crit3.jsonl
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
