#!/bin/bash
# Round 3 measurement evidence for bench.py's new legs: PMC passes (separate --pmc runs, kernel trace
# only) of the kernel each leg runs, at two launch sizes -> profiles/profile_<kernel>_<leg>.json fits
# (scripts/make_profile_json.py), then the bench line reading them and the rocprofv3 kernel stats of
# the same bench command.  Each GPU step has its own time limit; any failure ends the script.
#   f64        k_resident, config 2, f64 fixed, B=1024
#   adaptive   k_resident, config 2, f32 adaptive tol 1e-3, B=1024
#   config4    k_step (FUSED), config 4, f32 fixed, B=1024 (one launch per step: per-launch bytes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r03}
OUT=$ROOT/gpurun_out/round_$TAG
mkdir -p "$OUT/profile"
cp profiles/profile_k_onchip.json profiles/profile_k_resident.json "$OUT/profile/"
GROUPS_ALL="FETCH_SIZE|WRITE_SIZE|SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
prof() {  # prof NAME KERNEL DTYPE CONFIG MODE K1 K2 ENV...
    local name=$1 kern=$2 dtype=$3 config=$4 mode=$5 k1=$6 k2=$7; shift 7
    local args=()
    for steps in $k1 $k2; do
        env "$@" STEPS=$steps TAG=${TAG}_${name}_$steps PMC_GROUPS="$GROUPS_ALL" bash scripts/pmc.sh \
            > "$OUT/pmc_${name}_$steps.log" 2>&1 || { echo "pmc $name $steps failed"; tail -5 "$OUT/pmc_${name}_$steps.log"; return 1; }
        args+=("$steps:gpurun_out/pmc_${TAG}_${name}_$steps")
    done
    python scripts/make_profile_json.py $kern 1024 $dtype $config "$OUT/profile/profile_${kern}_${name}.json" mode=$mode "${args[@]}" > /dev/null
}
prof f64 k_resident f64 config2 fixed 10 30 ALG=2 DTYPE=f64 || exit 1
echo "f64 ok"
prof adaptive k_resident f32 config2 adaptive 5 15 ADAPTIVE=1 || exit 1
echo "adaptive ok"
prof config4 k_step f32 config4 fixed 2 4 CONFIG=config4 ALG=0 || exit 1
echo "config4 ok"
timeout -k 10 600 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} --profile-dir "$OUT/profile" > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" > "$OUT/bench.json"
echo "bench ok"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps ${STEPS:-20} --warmup ${WARMUP:-5} --no-cpu --profile-dir "$OUT/profile" \
    > "$OUT/rocprof.log" 2>&1 || { tail -20 "$OUT/rocprof.log"; exit 1; }
cd "$ROOT"
echo "rocprof ok"
