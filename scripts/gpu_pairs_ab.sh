#!/bin/bash
# A/B of k_onchip's wave-paired tiles (this tree) against a baseline build (expt/libbase.so):
# bench lines at the driver's 20 steps and at 200, each alternated twice.
set -eu
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
B="timeout -k 10 120 python bench.py --no-cpu --no-ab --no-inter --extra-batch 0"
for r in 1 2; do
  for st in "20 5" "200 50"; do
    set -- $st
    echo "new steps=$1 $($B --steps $1 --warmup $2 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["mean_launch_us"])')"
    echo "base steps=$1 $(ODESAT_LIB=$PWD/expt/libbase.so $B --steps $1 --warmup $2 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["mean_launch_us"])')"
  done
done
