#!/bin/bash
# Config 3 (k_wave: adaptive and fixed dt, B=1024) and the criterion shapes (hard.cnf, B=1, f64),
# product library vs expt/lib$VAR.so, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
one() { timeout -k 10 300 python scripts/bench_configs.py --configs config3,config3f ${CFG3_ARGS:-} --steps 200 --warmup 20 --no-cpu 2>/dev/null | python3 -c "
import sys,json
for line in sys.stdin:
    d=json.loads(line); print(d['config'] if 'config' in d else '', d.get('algorithm'), round(d['replica_steps_per_s']/1e6,2), 'M', round(d['ms_per_step'],5))"; }
crit() { timeout -k 10 300 python scripts/bench_criterion.py --calls 3 --no-cpu 2>/dev/null | tail -2; }
for r in 1 2; do
  echo "== prod"; one || exit 1; crit || exit 1
  echo "== $VAR"; ODESAT_LIB=$PWD/expt/lib$VAR.so one || exit 1; ODESAT_LIB=$PWD/expt/lib$VAR.so crit || exit 1
done
