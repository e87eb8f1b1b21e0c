#!/bin/bash
# A/B: the product build against expt/lib$OLD.so (default libold: the previous commit's build), the
# driver's 20-step line and the 200-step line, headline + adaptive legs, alternated; then the GPU
# parity suites on the product build (TESTS=1).
set -u
cd "$(dirname "$0")/.."
OLD=${OLD:-old}
B="timeout -k 10 150 python bench.py --no-cpu --only ${LEGS_ONLY:-adaptive} --extra-batch 0"
val() { python -c 'import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1]); a=d.get("adaptive",{})
f=d.get("f64",{}); ab=d.get("ab_hbm_streaming",{}); print("ab %.4g" % ab.get("value",0), "%.4g" % d["value"], "%.1f" % d["roofline"]["mean_launch_us"], "ada %.4g" % a.get("value",0), "f64 %.4g" % f.get("value",0))'; }
for r in 1 2 3; do
  for st in "20 5" "200 50"; do
    set -- $st
    o=$($B --steps $1 --warmup $2 2>/dev/null) || { echo "prod failed"; exit 1; }
    echo "new steps=$1 $(echo "$o" | val)"
    o=$(ODESAT_LIB=$PWD/expt/lib$OLD.so $B --steps $1 --warmup $2 2>/dev/null) || { echo "old failed"; exit 1; }
    echo "$OLD steps=$1 $(echo "$o" | val)"
  done
done
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py -x -q \
      --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log; exit $rc
fi
