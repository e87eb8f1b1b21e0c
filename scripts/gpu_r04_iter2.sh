#!/bin/bash
# Round 4, second A/B: split barriers with a tight poll (no s_sleep) for the fixed and the adaptive kernel
# against the default build (adaptive only, s_sleep 1); the config-4 owner-TT A/B.  Digests first.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r04j}
mkdir -p "$OUT"
for v in sbdef sbfix0 sbada0; do
  for mode in "" "--adaptive --steps 50"; do
    ODESAT_LIB=$PWD/expt/lib$v.so timeout -k 10 300 python -u scripts/state_digest.py --batch 256 --calls 3 $mode \
        > "$OUT/digest_${v}_${#mode}.jsonl" 2>"$OUT/digest_$v.err" || { echo "digest $v failed"; tail -3 "$OUT/digest_$v.err"; exit 1; }
  done
done
for m in 0 21; do
  for v in sbfix0 sbada0; do
    diff -q "$OUT/digest_sbdef_$m.jsonl" "$OUT/digest_${v}_$m.jsonl" || { echo "DIGESTS DIFFER $v $m"; cat "$OUT"/digest_*_$m.jsonl; exit 1; }
  done
done
echo "digests equal"
B="timeout -k 10 200 python -u bench.py --no-cpu --steady-calls 8 --skip f64,f64_adaptive,config3,inter,config4,config5,extra,ab"
val() { python -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][-1]); a=d["adaptive"]; print(round(d["value"]/1e6,3), round(d["roofline"]["mean_launch_us"],1), round(d["steady_state"]["value"]/1e6,3), round(d["steady_state"]["kernel_us_per_call"],1), "ada", round(a["value"]/1e6,3), round(a["roofline"]["mean_launch_us"],1))'; }
for r in 1 2; do
  for v in sbdef sbfix0 sbada0; do
    for st in "20 5" "200 50"; do
      set -- $st
      echo "$v steps=$1 $(ODESAT_LIB=$PWD/expt/lib$v.so $B --steps $1 --warmup $2 2>/dev/null | val)" || exit 1
    done
  done
done
c4() { python -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][-1]); print({k: d[k] for k in d if k in ("replica_steps_per_s","ms_per_step","mean_launch_us","value","kernel_ms_per_step","gpu_ms_per_step")})'; }
for i in 1 2; do for tt in 1 0; do
  echo "config4 tt=$tt $(ODESAT_FUSED_TT=$tt timeout -k 10 200 python -u scripts/bench_configs.py --configs config4 --steps 20 --warmup 5 --no-cpu 2>/dev/null | tee -a $OUT/config4_tt$tt.jsonl | c4)" || exit 1
done; done
echo done
