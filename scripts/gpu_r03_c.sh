# round 3: k_solo team sweep, config-4 row-gather ceiling, config-5 per-rank slices.  Each GPU step
# has its own limit; any non-zero status ends the script.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/solo_sweep.py > gpurun_out/solo_sweep.jsonl 2>&1 || { echo "sweep rc=$?"; tail -5 gpurun_out/solo_sweep.jsonl; exit 1; }
echo "sweep ok"
hipcc --offload-arch=gfx950 -O3 -o gpurun_out/row_ceiling scripts/micro/row_ceiling.hip || exit 1
timeout -k 10 120 ./gpurun_out/row_ceiling > gpurun_out/row_ceiling.jsonl 2>&1 || { echo "ceiling rc=$?"; cat gpurun_out/row_ceiling.jsonl; exit 1; }
cat gpurun_out/row_ceiling.jsonl
timeout -k 10 600 python -u scripts/partition_slices.py > gpurun_out/partition_slices.jsonl 2>&1 || { echo "slices rc=$?"; tail -5 gpurun_out/partition_slices.jsonl; exit 1; }
echo "slices ok"
