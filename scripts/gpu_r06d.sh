#!/bin/bash
# Round 6: k_onchip's adaptive step on the interleaved (y, h) layout (onchip.hpp ONCHIP_ADA_IL): the GPU
# suite on the product build (IL), then an A/B against the previous layout in the adaptive leg's shape,
# then PMC per pass of the IL build (scripts/gpu_r06c.sh part C).
set -u -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r06d}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu suite failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
A="--lib expt/libadanoil.so" B="--lib expt/libadail.so" ROUNDS=3 FIELD=adaptive \
    CMD="python bench.py --no-cpu --only adaptive --steady-calls 0 --steps 20 --warmup 5" \
    bash scripts/gpu_ab.sh | tee "$OUT/ab_il.txt" || exit 1
SWEEP=0 SPL=0 TAG=${TAG:-r06d} bash scripts/gpu_r06c.sh
