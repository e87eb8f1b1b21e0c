#!/bin/bash
set -u
cd "$(dirname "$0")/.."
for nl in ${LANES:-256}; do
  ODESAT_SOLO_LANES=$nl ODESAT_LIB=$PWD/expt/libstamps.so timeout -k 10 120 python -u scripts/solo_stamps.py 2>/dev/null || exit 1
done
