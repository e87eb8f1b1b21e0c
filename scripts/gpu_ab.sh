#!/bin/bash
# A/B of two configurations on one GPU box, alternated ROUNDS times: each is either bench.py options
# ("--lib expt/libNAME.so", "--knob K=V") or an environment string for scripts/tooling.py
# (XP_LIB=expt/libNAME.so from scripts/build_variant.sh, XP_KNOBS="K=V,...") and both run the same command, by default the driver-shaped headline (bench.py --steps 20 --warmup 5
# without the extra legs).  One line per run: the label and the bench value / kernel microseconds.
#   A="" B="XP_LIB=$PWD/expt/libX.so" [ROUNDS=3] [CMD="python bench.py ..."] bash scripts/gpu_ab.sh
# VTESTS=1 then runs the GPU parity and fuzz suites against B's library.
set -u
cd "$(dirname "$0")/.."
CMD=${CMD:-"python bench.py --no-cpu --only headline --steady-calls 0 --steps 20 --warmup 5"}
# FIELD: the legs whose value and kernel time to print, space-separated (default the headline)
val() { python scripts/ab_value.py; }
for r in $(seq 1 "${ROUNDS:-3}"); do
    for side in A B; do
        cfg=${!side:-}
        if [[ "$cfg" == --* ]]; then  # bench.py options (--lib PATH, --knob K=V)
            out=$(timeout -k 10 300 $CMD $cfg 2>/dev/null) || { echo "$side failed"; exit 1; }
        else  # an environment for scripts/tooling.py (bench.py reads neither XP_LIB nor XP_KNOBS: use --lib / --knob)
            if [[ -n "$cfg" && "$CMD" == *bench.py* ]]; then echo "$side: bench.py takes --lib / --knob, not [$cfg]"; exit 1; fi
            out=$(env $cfg timeout -k 10 300 $CMD 2>/dev/null) || { echo "$side failed"; exit 1; }
        fi
        echo "$side [$cfg] $(echo "$out" | val)"
    done
done
if [ "${VTESTS:-0}" = 1 ]; then
    lib=$(echo "${B:-}" | sed -n 's/.*XP_LIB=\([^ ]*\).*/\1/p')
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 200 \
        --timeout-method thread -p no:cacheprovider ${lib:+--odesat-lib $lib} 2>&1 | tail -2
fi
