#!/bin/bash
# One GPU session producing a round's evidence: parity tests, smoke, PMC HBM traffic of the two
# persistent kernels (separate --pmc passes, kernel-trace only), the bench line (reading that
# traffic), and the rocprofv3 kernel stats of the same bench command.  Each GPU step has its own
# time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r01}
OUT=$ROOT/gpurun_out/round_$TAG
mkdir -p "$OUT/traffic"
run() {  # run NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
    return $rc
}
STEPS=${STEPS:-50}
if [ "${TESTS:-1}" = 1 ]; then
    run pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -ra || exit $?
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
for k in onchip:3 resident:2; do
    name=${k%%:*}; alg=${k##*:}
    ALG=$alg STEPS=$STEPS TAG=${TAG}_$name PMC_GROUPS="FETCH_SIZE|WRITE_SIZE" bash scripts/pmc.sh > "$OUT/pmc_$name.log" 2>&1 \
        || { echo "pmc $name failed"; tail -5 "$OUT/pmc_$name.log"; exit 1; }
    python scripts/make_traffic.py gpurun_out/pmc_${TAG}_$name k_$name 1024 $STEPS f32 config2 \
        "$OUT/traffic/traffic_k_$name.json" || exit 1
done
run bench 900 python bench.py --traffic-dir "$OUT/traffic" || exit $?
grep '^{' "$OUT/bench.log" > "$OUT/bench.json"
export TMPDIR=/tmp
cd /tmp
run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --no-cpu --extra-batch 0 --traffic-dir "$OUT/traffic" || exit $?
cd "$ROOT"
find "$OUT/rocprof" -name '*kernel_stats.csv' -exec cat {} \;
