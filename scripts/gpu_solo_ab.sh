#!/bin/bash
# criterion benches, the product build against expt/lib$VAR.so, alternated
set -u
cd "$(dirname "$0")/.."
for r in 1 2; do
  for lib in prod ${VARS:-}; do
    if [ $lib = prod ]; then L=""; else L="ODESAT_LIB=$PWD/expt/lib$lib.so"; fi
    echo "== $lib"; env $L timeout -k 10 300 python -u scripts/bench_criterion.py --no-cpu --calls 3 2>/dev/null || exit 1
  done
done
