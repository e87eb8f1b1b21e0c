#!/bin/bash
# A round's measurement evidence in one GPU session (TAG names it, default r04):
#   * PMC fits (separate --pmc passes, kernel trace only; scripts/pmc.sh) of every bench leg's kernel
#     at two launch sizes -> profile_<kernel>[_variant].json (scripts/make_profile_json.py);
#   * the driver-shaped bench line (--steps 20 --warmup 5) reading those fits;
#   * the rocprofv3 kernel stats of the same bench command (the average launch duration per kernel,
#     to set beside the line's HIP-event launch times).
# Set SKIP_TESTS=0 to run the GPU suite and smoke() first; ONLY="name ..." to profile a subset.
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r04}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT/profile"
cp profiles/profile_*.json "$OUT/profile/"
if [ "${SKIP_TESTS:-1}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      > "$OUT/pytest_gpu.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
GROUPS_ALL="FETCH_SIZE|WRITE_SIZE|SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
want() { [ -z "${ONLY:-}" ] || [[ " $ONLY " == *" $1 "* ]]; }
prof() {  # prof NAME KERNEL DTYPE MODE CONFIG OUTFILE K1 K2 ENV...
    local name=$1 kern=$2 dtype=$3 mode=$4 config=$5 outf=$6 k1=$7 k2=$8; shift 8
    want "$name" || return 0
    local args=()
    for steps in $k1 $k2; do
        env "$@" CONFIG=$config STEPS=$steps TAG=${TAG}_${name}_$steps PMC_GROUPS="$GROUPS_ALL" bash scripts/pmc.sh \
            > "$OUT/pmc_${name}_$steps.log" 2>&1 || { echo "pmc $name $steps failed"; tail -5 "$OUT/pmc_${name}_$steps.log"; return 1; }
        args+=("$steps:gpurun_out/pmc_${TAG}_${name}_$steps")
    done
    python scripts/make_profile_json.py $kern 1024 $dtype $config "$OUT/profile/$outf" mode=$mode "${args[@]}" > /dev/null \
        || { echo "fit $name failed"; return 1; }
    echo "pmc $name ok"
}
prof onchip k_onchip f32 fixed config2 profile_k_onchip.json 10 50 || exit 1
prof onchip_ada k_onchip f32 adaptive config2 profile_k_onchip_adaptive.json 5 15 ADAPTIVE=1 || exit 1
prof res_f64 k_resident f64 fixed config2 profile_k_resident_f64.json 10 30 ALG=2 DTYPE=f64 || exit 1
prof res_f64_ada k_resident f64 adaptive config2 profile_k_resident_f64_adaptive.json 5 15 ALG=2 DTYPE=f64 ADAPTIVE=1 || exit 1
prof res k_resident f32 fixed config2 profile_k_resident.json 10 50 ALG=2 || exit 1
prof wave_c3 k_wave f32 adaptive config3 profile_k_wave.json 20 100 ADAPTIVE=1 || exit 1
prof step_c4 k_step f32 fixed config4 profile_k_step_config4.json 2 4 || exit 1  # one launch per step: per-dispatch means
if want part; then  # config 5's partitioned step at world 1: per-kernel counter bytes per step
  pargs=()
  for mode in clauses variables; do
    PROG=scripts/bench_partition.py PROG_ARGS="--config config5 --mode $mode --steps 20 --warmup 5 --graph 0" \
      TAG=${TAG}_part_$mode PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum" bash scripts/pmc.sh \
      > "$OUT/pmc_part_$mode.log" 2>&1 || { echo "pmc part $mode failed"; tail -5 "$OUT/pmc_part_$mode.log"; exit 1; }
    pargs+=("$mode:gpurun_out/pmc_${TAG}_part_$mode")
  done
  python scripts/make_part_profile.py "$OUT/profile/profile_k_part_config5.json" "${pargs[@]}" > /dev/null \
      || { echo "fit part failed"; exit 1; }
  echo "pmc part ok"
fi
if want bench; then
  timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --profile-dir "$OUT/profile" > "$OUT/bench.log" 2>&1 \
      || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
  grep '^{' "$OUT/bench.log" > "$OUT/bench.json"; echo "bench ok"
fi
if want rocprof; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu --profile-dir "$OUT/profile" \
      > "$OUT/rocprof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/rocprof.log"; exit 1; }
  echo "rocprof ok"
  cd "$ROOT"
fi
echo done
