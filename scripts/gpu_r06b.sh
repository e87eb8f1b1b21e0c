#!/bin/bash
# Round 6: the YG variant of the f64 adaptive k_resident -- its parity tests, then an A/B against the
# stored-mn kernel (knob RES_YG = 0) in the f64_adaptive leg's shape, alternated on one box.
set -u -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r06b}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest "tests/test_gpu_parity.py::test_resident_f64_register_tiles_match_streaming_and_oracle" \
    "tests/test_gpu_configs.py::test_config2_bench_leg_kernels_bitexact" -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/targeted.log" 2>&1 || { echo targeted failed; tail -30 "$OUT/targeted.log"; exit 1; }
tail -3 "$OUT/targeted.log"
A="--knob RES_YG=0" B="" ROUNDS=${ROUNDS:-3} FIELD="f64_adaptive" \
    CMD="python bench.py --no-cpu --only f64_adaptive --steady-calls 0 --steps 20 --warmup 5" \
    bash scripts/gpu_ab.sh 2>&1 | tee "$OUT/ab_yg.txt"
