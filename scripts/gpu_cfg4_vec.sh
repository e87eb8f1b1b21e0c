#!/bin/bash
# Config 4 FUSED with 1 / 2 / 4 contiguous replicas per lane (W = 64 / 128 / 256; ODESAT_VEC).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in 1 2 4 1 2 4; do
  echo "VEC=$v $(ODESAT_VEC=$v timeout -k 10 300 python scripts/bench_configs.py --configs config4 --steps 30 --warmup 3 --no-cpu 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['algorithm'], round(d['ms_per_step'],4), round(d['algorithmic_GBps']))")" || exit 1
done
