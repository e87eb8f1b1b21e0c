# round 3: adaptive k_onchip parity + its bench leg, then the k_solo sweep, config-4 row-gather
# ceiling and config-5 per-rank slices.  Each GPU step has its own limit; a fault ends the script.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "onchip or algorithms_identical or wave_teams" > gpurun_out/t4.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/t4.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --only adaptive --no-cpu > gpurun_out/b4.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/b4.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/b4.log') if l.startswith('{')][0]); a=d['adaptive']; print('adaptive', a['value'], a['ms_per_step'], a['kernel'])"
timeout -k 10 300 python -u scripts/solo_sweep.py > gpurun_out/solo_sweep.jsonl 2>&1 || { echo "sweep rc=$?"; tail -5 gpurun_out/solo_sweep.jsonl; exit 1; }
echo "sweep ok"
hipcc --offload-arch=gfx950 -O3 -o gpurun_out/row_ceiling scripts/micro/row_ceiling.hip || exit 1
timeout -k 10 120 ./gpurun_out/row_ceiling > gpurun_out/row_ceiling.jsonl 2>&1 || { echo "ceiling rc=$?"; cat gpurun_out/row_ceiling.jsonl; exit 1; }
cat gpurun_out/row_ceiling.jsonl
timeout -k 10 600 python -u scripts/partition_slices.py > gpurun_out/partition_slices.jsonl 2>&1 || { echo "slices rc=$?"; tail -5 gpurun_out/partition_slices.jsonl; exit 1; }
echo "slices ok"
