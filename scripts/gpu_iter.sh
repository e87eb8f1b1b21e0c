#!/bin/bash
# One iteration on the GPU box: parity tests, bench (default algorithm + A/B), kernel stats.
# Each GPU step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/iter
mkdir -p "$OUT"
run() {  # run NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -4 "$OUT/$name.log"
    return $rc
}
if [ "${TESTS:-1}" = 1 ]; then
    run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -ra || exit $?
fi
run bench 600 python bench.py --no-cpu ${BENCH_ARGS:-} || exit $?
if [ -n "${AB:-}" ]; then
    run bench_ab 600 python bench.py --no-cpu --extra-batch 0 --alg $AB || exit $?
fi
if [ "${PROF:-1}" = 1 ]; then
    export TMPDIR=/tmp
    cd /tmp
    run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" --no-cpu --extra-batch 0 || exit $?
    cd "$ROOT"
    find "$OUT/rocprof" -name '*kernel_stats.csv' -exec cat {} \;
fi
