#!/bin/bash
# Round-2 GPU check: the whole -m gpu suite, then a short bench line.  Each GPU step has its own
# time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20.log 2>&1 || { tail -20 gpurun_out/bench20.log; exit 1; }
tail -1 gpurun_out/bench20.log
if [ "${LONG:-0}" = 1 ]; then
    timeout -k 10 600 python bench.py --steps 200 --warmup 50 --no-cpu > gpurun_out/bench200.log 2>&1 || { tail -20 gpurun_out/bench200.log; exit 1; }
    tail -1 gpurun_out/bench200.log
fi
