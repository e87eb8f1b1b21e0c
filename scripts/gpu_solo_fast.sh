#!/bin/bash
# k_solo_fast -- parity suites (fuzz: every path, k_solo general and fast), then the criterion
# benches, the product against the previous build (expt/libold.so), alternated, and a lane sweep.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py tests/test_gpu_parity.py \
    tests/test_boundary.py tests/test_gpu_runs.py -k "solo or wave or criterion or boundary or unbounded or fuzz" > gpurun_out/solo_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/solo_tests.log; exit 1; }
tail -2 gpurun_out/solo_tests.log
for r in 1 2; do
  echo "== new"; timeout -k 10 300 python -u scripts/bench_criterion.py --no-cpu 2>/dev/null || exit 1
  echo "== old"; ODESAT_LIB=$PWD/expt/libold.so timeout -k 10 300 python -u scripts/bench_criterion.py --no-cpu 2>/dev/null || exit 1
done
for nl in ${SWEEP:-}; do
  echo "== lanes $nl"; ODESAT_SOLO_LANES=$nl timeout -k 10 300 python -u scripts/bench_criterion.py --no-cpu --calls 3 2>/dev/null || exit 1
done
