#!/bin/bash
# A/B of the product build against expt/lib$VAR.so (bench lines, alternated), then the variant's
# ONCHIP parity tests (VTESTS=1).
set -u
cd "$(dirname "$0")/.."
B="timeout -k 10 120 python bench.py --no-cpu --no-ab --no-inter --extra-batch 0"
val() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["mean_launch_us"])'; }
for r in 1 2; do
  for st in "200 50" "20 5"; do
    set -- $st
    echo "prod steps=$1 $($B --steps $1 --warmup $2 | val)" || exit 1
    echo "$VAR steps=$1 $(ODESAT_LIB=$PWD/expt/lib$VAR.so $B --steps $1 --warmup $2 | val)" || exit 1
  done
done
if [ "${VTESTS:-0}" = 1 ]; then
  ODESAT_LIB=$PWD/expt/lib$VAR.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
fi
