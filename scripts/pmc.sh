#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only -- no sys/runtime trace with --pmc).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_${TAG:-x}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
PMC_GROUPS=${PMC_GROUPS:-"FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum|TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum|GRBM_GUI_ACTIVE SQ_WAVES"}
IFS='|' read -ra GLIST <<< "$PMC_GROUPS"
for grp in "${GLIST[@]}"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
        python3 "$ROOT/${PROG:-scripts/prof_step.py}" ${PROG_ARGS:-} > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($grp) failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
    echo "pass $i ($grp) ok"
done
