#!/bin/bash
# k_onchip timing experiments: bench lines (100-step launches, B = 1024) of the product library and of
# expt/lib<NAME>.so variants (EXPTS), then the stamp reader on the stamp variants (STAMPS).  Each GPU
# step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for e in base ${EXPTS:-}; do
  if [ $e = base ]; then L=""; else L="ODESAT_LIB=$PWD/expt/lib$e.so"; fi
  env $L timeout -k 10 120 python bench.py --no-cpu --extra-batch 0 --no-ab --no-inter --steps ${STEPS:-100} --warmup 5 \
      > gpurun_out/expt_$e.log 2>&1 || { echo "$e failed"; tail -3 gpurun_out/expt_$e.log; exit 1; }
  echo "$e $(grep -o '"value": [0-9.]*' gpurun_out/expt_$e.log | head -1) $(grep -o '"mean_launch_us": [0-9.]*' gpurun_out/expt_$e.log)"
done
done
for e in ${STAMPS:-}; do
  echo "== stamps $e"
  ODESAT_LIB=$PWD/expt/lib$e.so timeout -k 10 120 python scripts/onchip_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
done
