# round 3: k_solo with one barrier for the unsat vote and the lazy dt update -- parity, criterion.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py tests/test_gpu_parity.py \
    -k "solo or wave or criterion" > gpurun_out/solo_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/solo_tests.log; exit 1; }
tail -2 gpurun_out/solo_tests.log
timeout -k 10 300 python -u scripts/bench_criterion.py > gpurun_out/crit4.jsonl 2>&1 || { echo "crit failed"; tail -5 gpurun_out/crit4.jsonl; exit 1; }
cat gpurun_out/crit4.jsonl
