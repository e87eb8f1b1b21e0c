#!/bin/bash
# k_wave (small instances): the GPU parity tests that run it, then config 3 throughput.  Each GPU step
# has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/wave; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "${PYTEST_K:-wave or config3 or golden or inter or small or hard or easy or adaptive}" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for team in ${TEAMS:-2 1}; do
    ODESAT_WAVE_TEAM=$team timeout -k 10 600 python scripts/bench_configs.py --configs config3 --no-cpu > $OUT/config3_t$team.jsonl 2> $OUT/config3.err || { tail -20 $OUT/config3.err; exit 1; }
    python3 - $OUT/config3_t$team.jsonl $team <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print("team", sys.argv[2], d["workload"], d["batch"], round(d["replica_steps_per_s"] / 1e6, 2), "M", round(d["ms_per_step"], 4), "ms")
PY
done
