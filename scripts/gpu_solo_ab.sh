#!/bin/bash
# A/B of the product build against expt/lib$VAR.so on the reference's criterion benches
# (scripts/bench_criterion.py, hard.cnf, B = 1, f64), alternated, then the solo parity tests
# (TESTK: their -k filter; VTEST=1: on the variant's library).
set -u
cd "$(dirname "$0")/.."
o=gpurun_out/${TAG:-solo_ab}; mkdir -p $o
for r in 1 2 3; do
  timeout -k 10 120 python scripts/bench_criterion.py --no-cpu --calls 5 | sed "s/^/prod /" >> $o/ab.txt || exit 1
  ODESAT_LIB=$PWD/expt/lib$VAR.so timeout -k 10 120 python scripts/bench_criterion.py --no-cpu --calls 5 | sed "s/^/$VAR /" >> $o/ab.txt || exit 1
done
L=""; [ "${VTEST:-0}" = 1 ] && L=$PWD/expt/lib$VAR.so
ODESAT_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_runs.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "${TESTK:-solo}" > $o/pytest.log 2>&1; echo "pytest rc=$?" >> $o/pytest.log
cat $o/ab.txt; tail -2 $o/pytest.log
