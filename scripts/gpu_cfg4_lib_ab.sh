#!/bin/bash
# Config 4 (FUSED) with the product library and with expt/lib$VAR.so, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
one() { timeout -k 10 300 python scripts/bench_configs.py --configs config4 --steps 30 --warmup 3 --no-cpu 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['algorithm'], round(d['ms_per_step'],4), round(d['algorithmic_GBps']))"; }
for r in 1 2; do
  echo "prod $(one)" || exit 1
  echo "$VAR $(ODESAT_LIB=$PWD/expt/lib$VAR.so one)" || exit 1
done
