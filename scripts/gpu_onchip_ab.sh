#!/bin/bash
# k_onchip A/B: the ONCHIP parity tests, then bench lines (20- and 200-step launches) with the
# persistent replica loop on and off.  Each GPU step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/onchip_ab; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "${PYTEST_K:-onchip or config2 or boundary or inter or continue}" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
for p in ${MODES:-1 0}; do
    for st in 20 200; do
        ODESAT_ONCHIP_PERSIST=$p timeout -k 10 300 python bench.py --steps $st --warmup 5 --no-cpu --no-ab --no-inter --extra-batch 256 \
            > $OUT/b_${p}_${st}.log 2>&1 || { tail -20 $OUT/b_${p}_${st}.log; exit 1; }
        tail -1 $OUT/b_${p}_${st}.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('persist=$p steps=$st', round(d['value']/1e6,3), 'M', round(d['ms_per_step']*1e3,2), 'us/step', 'B256', round(d['extra_batch']['value']/1e6,3))"
    done
done
done
