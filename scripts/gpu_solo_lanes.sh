set -u
for r in 1 2; do
for nl in 128 192 256; do
  echo "== lanes $nl"; ODESAT_SOLO_LANES=$nl timeout -k 10 300 python -u scripts/bench_criterion.py --no-cpu --calls 3 2>/dev/null || exit 1
done
done
