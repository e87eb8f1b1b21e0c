#!/bin/bash
# One GPU session producing the round's evidence: parity tests, smoke, bench, rocprofv3 kernel
# stats of the same bench command, PMC traffic of the dominant kernel.  Each GPU step has its own
# time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r01}
OUT=$ROOT/gpurun_out/round_$TAG
mkdir -p "$OUT"
run() {  # run NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
    return $rc
}
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -ra || exit $?
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 900 python bench.py || exit $?
grep '^{' "$OUT/bench.log" > "$OUT/bench.json"
export TMPDIR=/tmp
cd /tmp
run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --no-cpu --extra-batch 0 || exit $?
cd "$ROOT"
TAG=${TAG}_pmc PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum|TCC_HIT_sum TCC_MISS_sum" \
    STEPS=20 bash scripts/pmc.sh || exit $?
python scripts/make_traffic.py gpurun_out/pmc_${TAG}_pmc k_resident 1024 20 f32 config2 "$OUT/traffic.json"
