#!/bin/bash
# k_solo: short arithmetic on in-range states + one-barrier vote -- parity suites, then the criterion
# benches: product (FAST), product with ODESAT_SOLO_FAST=0 (the vote change alone), the previous build.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py tests/test_gpu_parity.py \
    tests/test_boundary.py tests/test_gpu_runs.py -k "solo or wave or criterion or boundary or unbounded" > gpurun_out/solo_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/solo_tests.log; exit 1; }
tail -2 gpurun_out/solo_tests.log
for r in 1 2; do
  echo "== fast"; timeout -k 10 300 python -u scripts/bench_criterion.py --no-cpu 2>/dev/null || exit 1
  echo "== fast0"; ODESAT_SOLO_FAST=0 timeout -k 10 300 python -u scripts/bench_criterion.py --no-cpu 2>/dev/null || exit 1
  echo "== old"; ODESAT_LIB=$PWD/expt/libold.so timeout -k 10 300 python -u scripts/bench_criterion.py --no-cpu 2>/dev/null || exit 1
done
