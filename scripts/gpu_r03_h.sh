# round 3: PMC fit of the (branched) adaptive k_onchip, then the driver-shaped bench line.
set -u
mkdir -p gpurun_out
GROUPS_ALL="FETCH_SIZE|WRITE_SIZE|SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
args=()
for steps in 5 15; do
    ADAPTIVE=1 STEPS=$steps TAG=r03h_ocada_$steps PMC_GROUPS="$GROUPS_ALL" bash scripts/pmc.sh > gpurun_out/pmch_ocada_$steps.log 2>&1 \
        || { echo "pmc failed"; tail -5 gpurun_out/pmch_ocada_$steps.log; exit 1; }
    args+=("$steps:gpurun_out/pmc_r03h_ocada_$steps")
done
python scripts/make_profile_json.py k_onchip 1024 f32 config2 profiles/profile_k_onchip_adaptive.json mode=adaptive "${args[@]}" > /dev/null || exit 1
cp profiles/profile_k_onchip_adaptive.json gpurun_out/
echo "pmc ok"
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_h.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_h.log; exit 1; }
grep '^{' gpurun_out/bench_h.log > gpurun_out/bench_h.json; echo "bench ok"
