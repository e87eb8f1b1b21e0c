#!/bin/bash
# Round 4 iteration on the GPU: the whole GPU suite and smoke() on the product build, the split-barrier
# A/B (scripts/gpu_splitbar_ab.sh), the config-4 owner-TT A/B and the per-call fold A/B (ODESAT_CALL_FOLD).
# Each GPU step has its own time limit; a failing step ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r04i}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "suite failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
TAG=${TAG:-r04i}_sb bash scripts/gpu_splitbar_ab.sh || exit 1
for i in 1 2; do for tt in 1 0; do
  echo "config4 tt=$tt $(ODESAT_FUSED_TT=$tt timeout -k 10 200 python -u scripts/bench_configs.py --configs config4 --steps 20 --warmup 5 --no-cpu 2>/dev/null | tail -1 | cut -c1-220)" || exit 1
done; done
B="timeout -k 10 200 python -u bench.py --no-cpu --steady-calls 0 --only config3"
val() { python -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][-1]); c=d["config3"]; print(round(d["value"]/1e6,3), round(d["ms_per_step"]*1e3,2), round(d["roofline"]["mean_launch_us"],1), "config3", round(c["value"]/1e6,2), round(c["ms_per_step"]*1e3,2), round(c["roofline"]["mean_launch_us"],1))'; }
for i in 1 2; do for fold in 1 0; do
  echo "fold=$fold $(ODESAT_CALL_FOLD=$fold $B --steps 20 --warmup 5 2>/dev/null | val)" || exit 1
done; done
for i in 1 2; do for v in prod foldlate; do
  L=""; [ $v = prod ] || L="ODESAT_LIB=$PWD/expt/lib$v.so"
  echo "criterion $v $(env $L timeout -k 10 200 python -u scripts/bench_criterion.py --no-cpu 2>/dev/null | tr '\n' ' ')" || exit 1
done; done
echo done
