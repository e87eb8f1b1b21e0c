#!/bin/bash
# One GPU session producing a round's measurement evidence: PMC passes (separate --pmc runs, kernel
# trace only) of the two persistent kernels at two launch sizes -> profiles/profile_<kernel>.json fits,
# the bench line reading them, and the rocprofv3 kernel stats of the same bench command (its warmup
# launch as long as the timed one, so the kernel's rocprof average is the timed launch's length).  Each GPU
# step has its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r02}
OUT=$ROOT/gpurun_out/round_$TAG
mkdir -p "$OUT/profile"
run() {  # run NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
    return $rc
}
if [ "${TESTS:-0}" = 1 ]; then
    run pytest_gpu 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -ra || exit $?
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
GROUPS_ALL="FETCH_SIZE|WRITE_SIZE|SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for k in onchip:3 resident:2; do
    name=${k%%:*}; alg=${k##*:}
    args=()
    for steps in 10 50; do
        ALG=$alg STEPS=$steps TAG=${TAG}_${name}_$steps PMC_GROUPS="$GROUPS_ALL" bash scripts/pmc.sh \
            > "$OUT/pmc_${name}_$steps.log" 2>&1 || { echo "pmc $name $steps failed"; tail -5 "$OUT/pmc_${name}_$steps.log"; exit 1; }
        args+=("$steps:gpurun_out/pmc_${TAG}_${name}_$steps")
    done
    python scripts/make_profile_json.py k_$name 1024 f32 config2 "$OUT/profile/profile_k_$name.json" "${args[@]}" || exit 1
done
run bench 900 python bench.py --steps ${STEPS:-200} --warmup ${WARMUP:-50} --profile-dir "$OUT/profile" || exit $?
grep '^{' "$OUT/bench.log" > "$OUT/bench.json"
export TMPDIR=/tmp
cd /tmp
run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps ${STEPS:-200} --warmup ${STEPS:-200} --no-cpu --extra-batch 0 --no-inter \
    --profile-dir "$OUT/profile" || exit $?
cd "$ROOT"
find "$OUT/rocprof" -name '*kernel_stats.csv' -exec cat {} \;
