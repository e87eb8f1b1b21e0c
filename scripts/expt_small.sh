# A/B of experimental builds on the small-instance workloads (criterion benches, config 3)
set -u
for e in ${EXPTS:-base}; do
  if [ $e = base ]; then L=""; else L="ODESAT_LIB=$PWD/expt/lib$e.so"; fi
  env $L timeout -k 10 200 python scripts/bench_criterion.py --no-cpu > gpurun_out/small_$e.log 2>&1 || { echo "$e failed"; tail -3 gpurun_out/small_$e.log; exit 1; }
  env $L timeout -k 10 200 python scripts/bench_configs.py --configs config3,config3f --no-cpu >> gpurun_out/small_$e.log 2>&1 || exit 1
  echo "== $e"; grep "^{" gpurun_out/small_$e.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    print(d.get('bench', d.get('config')), round(d.get('gpu_ms_per_call', 0),1), round(d.get('replica_steps_per_s', 0)/1e6,1))"
done
