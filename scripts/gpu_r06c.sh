#!/bin/bash
# Round 6 measurements on one box (variants from scripts/build_variant.sh in expt/):
#  A. the f64 fixed register-tile sweep: RES_RC x RES_RC_DEPTH, the f64 leg's shape, alternated;
#  B. k_onchip's adaptive pass 2 on plain barriers (ONCHIP_SPLITBAR=0) against split ones, the adaptive leg;
#  C. PMC per pass of k_onchip's adaptive step: the full build and the builds without
#     pass 2 / pass 1 (ONCHIP_ADA_SKIP, timing-only), one counter group per rocprofv3 pass.
set -u -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r06c}
mkdir -p "$OUT"
if [ "${SWEEP:-1}" = 1 ]; then
for r in 1 2; do
    for v in ${RC_VARIANTS:-rc28d4 rc16d4 rc20d4 rc24d4 rc18d6 rc24d6 rc16d8 rc24d8}; do
        out=$(timeout -k 10 300 python bench.py --no-cpu --only f64 --steady-calls 0 --steps 20 --warmup 5 \
              --lib expt/lib$v.so 2>/dev/null) || { echo "$v failed"; exit 1; }
        echo "$v $(echo "$out" | FIELD=f64 python scripts/ab_value.py)" | tee -a "$OUT/rc_sweep.txt"
    done
done
fi
if [ "${SPL:-1}" = 1 ]; then
A="--lib expt/libonchipctl.so" B="--lib expt/libspl0.so" ROUNDS=3 FIELD=adaptive \
    CMD="python bench.py --no-cpu --only adaptive --steady-calls 0 --steps 20 --warmup 5" \
    bash scripts/gpu_ab.sh | tee "$OUT/ab_spl0.txt" || exit 1
fi
if [ "${PMC:-1}" = 1 ]; then
for v in onchipctl adaskip1 adaskip2; do
    XP_LIB=$PWD/expt/lib$v.so ADAPTIVE=1 TAG=${TAG:-r06c}_$v \
    PMC_GROUPS="SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE|GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
        bash scripts/pmc.sh || exit 1
done
fi
echo done
