#!/bin/bash
set -u
cd "$(dirname "$0")/.."
for nl in 64 128 192 256 512; do
  ODESAT_SOLO_LANES=$nl ODESAT_LIB=$PWD/expt/libstamps.so timeout -k 10 120 python -u scripts/solo_stamps.py 2>/dev/null || exit 1
done
for nl in 64 128 192 256 512; do
  echo "== lanes $nl"; ODESAT_SOLO_LANES=$nl timeout -k 10 300 python -u scripts/bench_criterion.py --no-cpu --calls 3 2>/dev/null || exit 1
done
