#!/bin/bash
# A/B: 12-byte onchip records (expt/librec12.so) against the product build, then the onchip parity
# suites on the variant.
set -u
cd "$(dirname "$0")/.."
OLD=rec12 LEGS_ONLY=adaptive TESTS=0 bash scripts/gpu_ab_old_new.sh || exit 1
ODESAT_LIB=$PWD/expt/librec12.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/rec12_tests.log 2>&1; rc=$?; tail -2 gpurun_out/rec12_tests.log; exit $rc
