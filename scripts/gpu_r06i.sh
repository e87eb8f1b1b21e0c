#!/bin/bash
# Round 6: k_wave's partial-round tail launch (WAVE_TAIL): its parity tests, then config 3's adaptive
# step at batches around whole device rounds, with and without the tail launch.
set -u -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r06i}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "wave" -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/wave_tests.log" 2>&1 || { echo "wave tests failed"; tail -30 "$OUT/wave_tests.log"; exit 1; }
tail -2 "$OUT/wave_tests.log"
for r in 1 2; do
    for k in "" "--knob WAVE_TAIL=0"; do
        timeout -k 10 300 python -u scripts/batch_scaling.py --out "$OUT/tail_scaling.jsonl" --families config3:f32:adaptive,config3:f32:fixed \
            --batches ${BATCHES:-1024,1100,1280,1536,1792,2048} $k || exit 1
    done
done
