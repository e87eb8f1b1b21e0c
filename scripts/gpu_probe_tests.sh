set -u
timeout -k 10 300 python scripts/probe_headline.py || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_x.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu_x.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "== wave fast"; timeout -k 10 300 python scripts/bench_configs.py --configs config3,config3f --no-cpu 2>/dev/null | tail -4 || exit 1
  echo "== wave general"; ODESAT_WAVE_FAST=0 timeout -k 10 300 python scripts/bench_configs.py --configs config3,config3f --no-cpu 2>/dev/null | tail -4 || exit 1
done
