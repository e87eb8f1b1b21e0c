#!/bin/bash
# Round 6: the f64 adaptive k_resident's register tiles and ring (RES_RC_ADA x RES_RC_DEPTH_ADA) and the
# non-temporal memory stream (RES_NT, both f64 legs), variants from scripts/build_variant.sh in expt/,
# alternated twice on one box in the f64 legs' shape.
set -u -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r06f}
mkdir -p "$OUT"
for r in 1 2; do
    for v in ${VARIANTS:-adactl adarc8 adarc16 adarc8d8 adarc16d8 resnt}; do
        out=$(timeout -k 10 300 python bench.py --no-cpu --only f64,f64_adaptive --steady-calls 0 --steps 20 --warmup 5 \
              --lib expt/lib$v.so 2>/dev/null) || { echo "$v failed"; exit 1; }
        echo "$v $(echo "$out" | FIELD="f64 f64_adaptive" python scripts/ab_value.py)" | tee -a "$OUT/ada_sweep.txt"
    done
done
