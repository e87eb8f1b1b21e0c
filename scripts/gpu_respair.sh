#!/bin/bash
# RESIDENT with a barrier after odd tiles only (timing-only build expt/librespair.so, results race)
# against the product RESIDENT, config 2 B=1024 fixed steps; then k_onchip stamps (expt/libstamps2.so).
set -u
cd "$(dirname "$0")/.."
B="timeout -k 10 120 python bench.py --no-cpu --no-ab --no-inter --extra-batch 0 --alg resident --steps 100 --warmup 20"
for r in 1 2; do
  echo "resident base $($B | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["mean_launch_us"])')" || exit 1
  echo "resident pairs-timing $(ODESAT_LIB=$PWD/expt/librespair.so $B | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["mean_launch_us"])')" || exit 1
done
ODESAT_LIB=$PWD/expt/libstamps2.so STEPS=20 timeout -k 10 120 python scripts/onchip_stamps.py
