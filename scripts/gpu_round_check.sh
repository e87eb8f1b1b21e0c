#!/bin/bash
# One GPU session: targeted tests (T=...), the GPU suite, smoke(), the driver-shaped bench line, and
# (DIST=1) the same line under a world-1 RCCL process group (the harness cost of the collective).
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-check}
mkdir -p "$OUT"
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
    return $rc
}
if [ -n "${T:-}" ]; then
    step targeted 600 python -u -m pytest $T -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
fi
if [ "${SUITE:-1}" = 1 ]; then
    step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
if [ "${BENCH:-1}" = 1 ]; then
    step bench 900 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} || exit 1
    grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"
fi
if [ "${DIST:-0}" = 1 ]; then
    ODESAT_BENCH_DIST=1 step bench_dist 900 python -u bench.py --steps 20 --warmup 5 --only adaptive --no-cpu || exit 1
    grep '^{' "$OUT/bench_dist.log" | tail -1 > "$OUT/bench_dist.json"
fi
echo done
