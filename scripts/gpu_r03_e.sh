# round 3: the GPU suite, the k_solo sweep and criterion benches, the PMC fit of adaptive k_onchip,
# then the driver-shaped bench line.  Each GPU step has its own limit; a fault ends the script.
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -p no:cacheprovider \
    > gpurun_out/t5.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 gpurun_out/t5.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/solo_sweep.py > gpurun_out/solo_sweep2.jsonl 2>&1 || { echo "sweep rc=$?"; exit 1; }
timeout -k 10 300 python -u scripts/bench_criterion.py > gpurun_out/crit2.jsonl 2>&1 || { echo "crit rc=$?"; exit 1; }
cat gpurun_out/crit2.jsonl | grep '^{'
GROUPS_ALL="FETCH_SIZE|WRITE_SIZE|SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
args=()
for steps in 5 15; do
    ADAPTIVE=1 STEPS=$steps TAG=r03_ocada_$steps PMC_GROUPS="$GROUPS_ALL" bash scripts/pmc.sh > gpurun_out/pmc_ocada_$steps.log 2>&1 \
        || { echo "pmc failed"; tail -5 gpurun_out/pmc_ocada_$steps.log; exit 1; }
    args+=("$steps:gpurun_out/pmc_r03_ocada_$steps")
done
python scripts/make_profile_json.py k_onchip 1024 f32 config2 gpurun_out/profile_k_onchip_adaptive.json mode=adaptive "${args[@]}" > /dev/null || exit 1
echo "pmc ok"
