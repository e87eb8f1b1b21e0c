#!/bin/bash
# A/B of the product against the same build with $ENVAB set (bench lines, alternated).
set -u
cd "$(dirname "$0")/.."
B="timeout -k 10 120 python bench.py --no-cpu --no-ab --no-inter --extra-batch 0"
val() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["mean_launch_us"])'; }
for r in 1 2; do
  for st in "200 50" "20 5"; do
    set -- $st
    echo "prod steps=$1 $($B --steps $1 --warmup $2 | val)" || exit 1
    echo "$ENVAB steps=$1 $(env $ENVAB $B --steps $1 --warmup $2 | val)" || exit 1
  done
done
