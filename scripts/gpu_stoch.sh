set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_stoch.py > gpurun_out/stoch_tests.log 2>&1
timeout -k 10 120 python -u scripts/bench_stoch.py > gpurun_out/stoch_bench.log 2>&1
timeout -k 10 120 python -u scripts/bench_stoch.py --batch 256 >> gpurun_out/stoch_bench.log 2>&1
ODESAT_STOCH_WAVE=0 timeout -k 10 120 python -u scripts/bench_stoch.py --steps 200 >> gpurun_out/stoch_bench.log 2>&1
timeout -k 10 120 python -u scripts/bench_stoch.py --config config2 --batch 256 --steps 50 --cpu-steps 50 >> gpurun_out/stoch_bench.log 2>&1
