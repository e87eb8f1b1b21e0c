#!/bin/bash
# Round 3 (later session) evidence after the min-of-others rewrite, k_solo_fast and the f64 ring of 8:
# the GPU suite, then PMC fits (separate --pmc passes, kernel trace only) of k_onchip fixed and
# adaptive and k_resident f64 at two launch sizes, the driver-shaped bench line reading them, and the
# rocprofv3 kernel stats of the same bench command.  Any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r3b
mkdir -p "$OUT/profile"
cp profiles/profile_*.json "$OUT/profile/"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      > "$OUT/pytest_gpu.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
GROUPS_ALL="FETCH_SIZE|WRITE_SIZE|SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
prof() {  # prof NAME KERNEL DTYPE MODE OUTFILE K1 K2 ENV...
    local name=$1 kern=$2 dtype=$3 mode=$4 outf=$5 k1=$6 k2=$7; shift 7
    local args=()
    for steps in $k1 $k2; do
        env "$@" STEPS=$steps TAG=r3b_${name}_$steps PMC_GROUPS="$GROUPS_ALL" bash scripts/pmc.sh \
            > "$OUT/pmc_${name}_$steps.log" 2>&1 || { echo "pmc $name $steps failed"; tail -5 "$OUT/pmc_${name}_$steps.log"; return 1; }
        args+=("$steps:gpurun_out/pmc_r3b_${name}_$steps")
    done
    python scripts/make_profile_json.py $kern 1024 $dtype config2 "$OUT/profile/$outf" mode=$mode "${args[@]}" > /dev/null
    echo "pmc $name ok"
}
prof onchip k_onchip f32 fixed profile_k_onchip.json 10 50 || exit 1
prof onchip_ada k_onchip f32 adaptive profile_k_onchip_adaptive.json 5 15 ADAPTIVE=1 || exit 1
prof res_f64 k_resident f64 fixed profile_k_resident_f64.json 10 30 ALG=2 DTYPE=f64 || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --profile-dir "$OUT/profile" > "$OUT/bench.log" 2>&1 \
    || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" > "$OUT/bench.json"; echo "bench ok"
timeout -k 10 600 python -u bench.py --steps 200 --warmup 50 --no-cpu --only adaptive,f64 --profile-dir "$OUT/profile" > "$OUT/bench200.log" 2>&1 \
    || { echo "bench200 failed"; tail -20 "$OUT/bench200.log"; exit 1; }
grep '^{' "$OUT/bench200.log" > "$OUT/bench200.json"; echo "bench200 ok"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu --profile-dir "$OUT/profile" \
    > "$OUT/rocprof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/rocprof.log"; exit 1; }
echo "rocprof ok"
cd "$ROOT"
timeout -k 10 300 python -u scripts/bench_criterion.py > "$OUT/criterion.jsonl" 2>/dev/null || { echo "criterion failed"; exit 1; }
echo "criterion ok"
timeout -k 10 300 python -u scripts/bench_configs.py --configs config3,config3f --no-cpu > "$OUT/configs3.jsonl" 2>/dev/null || { echo "configs failed"; exit 1; }
echo "configs ok"
