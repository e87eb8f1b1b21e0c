set -u
for e in ${EXPTS:-base E1 E2 E3}; do
  if [ $e = base ]; then L=""; else L="ODESAT_LIB=$PWD/expt/lib$e.so"; fi
  env $L timeout -k 10 120 python bench.py --no-cpu --extra-batch 0 --steps 100 > gpurun_out/expt_$e.log 2>&1 || { echo "$e failed"; tail -3 gpurun_out/expt_$e.log; exit 1; }
  echo "$e $(grep -o '"value": [0-9.]*' gpurun_out/expt_$e.log) $(grep -o '"mean_launch_us": [0-9.]*' gpurun_out/expt_$e.log)"
done
