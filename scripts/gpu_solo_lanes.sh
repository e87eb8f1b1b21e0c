#!/bin/bash
# The criterion benches (scripts/bench_criterion.py, hard.cnf, B = 1, f64) at several k_solo_fast team
# widths (ODESAT_SOLO_LANES), twice each, interleaved.
set -u
o=gpurun_out/${TAG:-solo_lanes}; mkdir -p $o
for r in 1 2; do
  for nl in 128 192 256 320 384; do
    ODESAT_SOLO_LANES=$nl timeout -k 10 120 python scripts/bench_criterion.py --no-cpu --calls 5 | sed "s/^/lanes=$nl /" >> $o/lanes.txt || exit 1
  done
done
cat $o/lanes.txt
