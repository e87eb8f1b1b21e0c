# k_solo parity first (stop on a fault, not on a test failure), then the round-3 profiles.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "wave_teams or wave_workgroup or algorithms_identical" > gpurun_out/t3.log 2>&1
rc=$?
echo "solo tests rc=$rc"; tail -3 gpurun_out/t3.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_criterion.py --no-cpu > gpurun_out/crit_solo.jsonl 2>&1
rc=$?
echo "criterion rc=$rc"; cat gpurun_out/crit_solo.jsonl | tail -3
[ $rc -eq 0 ] || exit $rc
bash scripts/round3_profile.sh
