# round 3: f64 adaptive steps on k_resident with the full-step clone in HBM (VFG) -- parity, A/B
# against FUSED (ODESAT_RES_VFG=0), and the PMC fit for the bench leg's traffic.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "clone_in_hbm or default_layout or resident_widths_match_fused_w64 and hard" > gpurun_out/vfg_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/vfg_tests.log; exit 1; }
echo "tests ok"
for vfg in 1 0; do
    ODESAT_RES_VFG=$vfg timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --only f64_adaptive --no-cpu \
        > gpurun_out/vfg_ab_$vfg.log 2>&1 || { echo "bench vfg=$vfg failed"; tail -5 gpurun_out/vfg_ab_$vfg.log; exit 1; }
done
echo "ab ok"
args=()
for steps in 5 15; do
    DTYPE=f64 ADAPTIVE=1 STEPS=$steps TAG=r03i_rf64a_$steps PMC_GROUPS="FETCH_SIZE|WRITE_SIZE" bash scripts/pmc.sh > gpurun_out/pmci_$steps.log 2>&1 \
        || { echo "pmc failed"; tail -5 gpurun_out/pmci_$steps.log; exit 1; }
    args+=("$steps:gpurun_out/pmc_r03i_rf64a_$steps")
done
python scripts/make_profile_json.py k_resident 1024 f64 config2 gpurun_out/profile_k_resident_f64_adaptive.json mode=adaptive "${args[@]}" > /dev/null || exit 1
echo "pmc ok"
