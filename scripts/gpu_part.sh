#!/bin/bash
# GPU: parity tests + the config-5 partitioned-instance bench at world 1 (both partitions).
# Each GPU step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/part
mkdir -p $OUT
run() {  # run NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -4 "$OUT/$name.log"
    return $rc
}
if [ "${TESTS:-1}" = 1 ]; then
    run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -ra || exit $?
fi
run part_var 600 python scripts/bench_partition.py --config config5 --mode variables --steps 100 || exit $?
run part_cla 600 python scripts/bench_partition.py --config config5 --mode clauses --steps 100 || exit $?
run bench 600 python bench.py --no-cpu --extra-batch 0 --no-ab || exit $?
