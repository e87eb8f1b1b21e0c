# A/B of experimental variants (scripts/build_variant.sh) against the product build; parity subset per variant
set -u
EXPTS="${EXPTS:-base}" bash scripts/expt.sh || exit 1
for e in ${PARITY:-}; do
  ODESAT_LIB=$PWD/expt/lib$e.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k onchip -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/par_$e.log 2>&1
  echo "$e parity rc=$?"; tail -1 gpurun_out/par_$e.log
done
