#!/bin/bash
# One GPU session: the byte-counter calibration (scripts/micro/fetch_calib.hip, one --pmc pass per
# counter group, kernel trace only) and, with BENCH=1, the driver-shaped bench line followed by a
# process listing (what outlives bench.py's main() at N = 1).  Every GPU step has its own time limit.
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=gpurun_out/${TAG:-calib}
mkdir -p "$OUT/pmc"
export TMPDIR=/tmp
timeout -k 10 120 scripts/micro/fetch_calib > "$OUT/calib_plain.jsonl" || { echo "calib rc=$?"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum" \
           "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
        -d "$ROOT/$OUT/pmc/p$i" -o run -- "$ROOT/scripts/micro/fetch_calib") > "$OUT/pmc_p$i.log" 2>&1 \
        || { echo "pmc pass $i rc=$?"; tail -5 "$OUT/pmc_p$i.log"; exit 1; }
    echo "pmc pass $i ok"
done
python3 scripts/fetch_calib_report.py "$OUT/calib_plain.jsonl" "$OUT/pmc" "$OUT/calib.json" || exit 1
if [ "${BENCH:-0}" = 1 ]; then
    ps -eo pid,ppid,pgid,sid,stat,etimes,args > "$OUT/ps_before.txt"
    timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo "bench rc=$?"; exit 1; }
    sleep 2
    ps -eo pid,ppid,pgid,sid,stat,etimes,args > "$OUT/ps_after.txt"
    grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"
fi
echo done
