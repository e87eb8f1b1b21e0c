#!/bin/bash
# The driver's round-end sequence on the tree as it stands: the GPU suite, smoke(), then the default
# bench line (--steps 20 --warmup 5).
set -u
cd "$(dirname "$0")/.."
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/final_pytest_gpu.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/final_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/final_bench.log; exit 1; }
grep '^{' gpurun_out/final_bench.log | tail -1 > gpurun_out/final_bench.json
python -c 'import json; d=json.load(open("gpurun_out/final_bench.json")); print("headline", d["value"], "f64", d["f64"]["value"], "f64_ada", d["f64_adaptive"]["value"], "ada", d["adaptive"]["value"], "ab", d["ab_hbm_streaming"]["value"])'
