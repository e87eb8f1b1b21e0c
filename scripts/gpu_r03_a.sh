set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_partition.py tests/test_gpu_runs.py tests/test_gpu_configs.py::test_config5_partitioned_full_size_vs_oracle > gpurun_out/t2.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b2.log 2>&1
