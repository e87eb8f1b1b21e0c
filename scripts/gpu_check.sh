#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel-trace profile.  Every GPU step has its own
# time limit; a crash / abort / timeout ends the script (no further GPU work in this call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r01}
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -5 "$OUT/$name.log"
    return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }

if [ "${SKIP_TESTS:-0}" != 1 ]; then
    step pytest_gpu 1100 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -ra
    rc=$?; if fatal $rc; then exit $rc; fi
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
step bench 900 python bench.py ${BENCH_ARGS:-} || exit $?
grep '^{' "$OUT/bench.log" > "$OUT/bench_$TAG.json" || true
if [ "${SKIP_PROF:-0}" != 1 ]; then
    export TMPDIR=/tmp
    cd /tmp
    step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" --no-cpu --extra-batch 0 || exit $?
    find "$OUT/prof_$TAG" -name '*stats*' | head
fi
