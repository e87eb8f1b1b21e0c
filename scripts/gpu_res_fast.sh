#!/bin/bash
# A/B of k_resident's short forms (ODESAT_RES_FAST=1, the default) against its general arithmetic
# (ODESAT_RES_FAST=0) on bench.py's f64 legs, alternated, the 20- and 200-step lines; then the GPU
# parity suites (TESTS=1).
set -u
cd "$(dirname "$0")/.."
B="timeout -k 10 150 python bench.py --no-cpu --only f64,f64_adaptive --extra-batch 0"
val() { python -c 'import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1]); f=d.get("f64",{}); fa=d.get("f64_adaptive",{})
print("f64 %.4g" % f.get("value",0), f.get("kernel", f.get("config",{}).get("kernel","")), "f64_ada %.4g" % fa.get("value",0), fa.get("kernel", fa.get("config",{}).get("kernel","")))'; }
for r in 1 2 3; do
  for st in "20 5" "200 50"; do
    set -- $st
    for f in 1 0; do
      o=$(ODESAT_RES_FAST=$f $B --steps $1 --warmup $2 2>/dev/null) || { echo "bench failed"; exit 1; }
      echo "fast=$f steps=$1 $(echo "$o" | val)"
      [ $r = 1 ] && [ $1 = 20 ] && echo "$o" | tail -1 > gpurun_out/res_fast_$f.json
    done
  done
done
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py -x -q \
      --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/res_fast_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/res_fast_tests.log; exit $rc
fi
