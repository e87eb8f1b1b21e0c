#!/bin/bash
# Adaptive config 2 (RESIDENT's adaptive pass): expt/lib$BASE.so vs expt/lib$VAR.so, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
one() { timeout -k 10 300 python scripts/bench_configs.py --configs config2a --steps 50 --warmup 5 --no-cpu 2>/dev/null | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['config'], round(d['replica_steps_per_s']/1e6,3), 'M', round(d['ms_per_step'],4), 'ms', round(d['algorithmic_GBps']), 'GB/s')"; }
for r in 1 2; do
  echo "$BASE $(ODESAT_LIB=$PWD/expt/lib$BASE.so one)" || exit 1
  echo "$VAR $(ODESAT_LIB=$PWD/expt/lib$VAR.so one)" || exit 1
done
