#!/bin/bash
# Call-overhead probe sweep (scripts/probe_call_overhead.py): host gap, warm-up per call, RCCL group,
# then one HIP runtime + kernel trace of four calls (no counters).
set -e
out=gpurun_out/${TAG:-r04q}
mkdir -p $out
run() { env "$@" CALLS=${CALLS:-12} timeout -k 10 120 python -u scripts/probe_call_overhead.py 2>> $out/overhead_gap.err | grep '^{' >> $out/overhead_gap.jsonl; }
run DIST=1 WARM=1 BARRIER=1
run DIST=1 WARM=1 BARRIER=1 PREBAR=1
run DIST=1 BARRIER=1 PREBAR=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
CALLS=4 timeout -k 10 180 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $out/trace -o run -- python3 -u scripts/probe_call_overhead.py > $out/trace.log 2>&1
