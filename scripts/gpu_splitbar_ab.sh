#!/bin/bash
# Round 4: k_onchip split barriers (ONCHIP_SPLITBAR) against the same build without them
# (expt/libsplitbar.so vs expt/libnosplit.so, both -DONCHIP_ONLY_TR=90): bit-exactness (state digests of
# long runs, the config-2 parity test) and the headline timing, alternated.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-splitbar}
mkdir -p "$OUT"
for v in splitbar splitbar2 nosplit; do
  ODESAT_LIB=$PWD/expt/lib$v.so timeout -k 10 300 python -u scripts/state_digest.py --batch 256 --steps 200 --calls 3 \
      > "$OUT/digest_$v.jsonl" 2>"$OUT/digest_$v.err" || { echo "digest $v failed"; tail -3 "$OUT/digest_$v.err"; exit 1; }
done
if diff -q "$OUT/digest_splitbar.jsonl" "$OUT/digest_nosplit.jsonl" && diff -q "$OUT/digest_splitbar2.jsonl" "$OUT/digest_nosplit.jsonl"; then echo "digests equal"; else echo "DIGESTS DIFFER"; cat "$OUT"/digest_*.jsonl; exit 1; fi
for v in splitbar nosplit; do  # adaptive steps
  ODESAT_LIB=$PWD/expt/lib$v.so timeout -k 10 300 python -u scripts/state_digest.py --batch 256 --steps 50 --calls 3 --adaptive \
      > "$OUT/digest_ada_$v.jsonl" 2>"$OUT/digest_ada_$v.err" || { echo "digest ada $v failed"; tail -3 "$OUT/digest_ada_$v.err"; exit 1; }
done
if diff -q "$OUT/digest_ada_splitbar.jsonl" "$OUT/digest_ada_nosplit.jsonl"; then echo "adaptive digests equal"; else echo "ADAPTIVE DIGESTS DIFFER"; cat "$OUT"/digest_ada_*.jsonl; exit 1; fi
ODESAT_LIB=$PWD/expt/libsplitbar.so timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_config2_full_size_subset_bitexact_and_properties[None]" \
    "tests/test_gpu_configs.py::test_config2_bench_leg_kernels_bitexact[adaptive-f32-True-k_onchip]" \
    -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/parity.log" 2>&1 || { echo "parity failed"; tail -20 "$OUT/parity.log"; exit 1; }
tail -1 "$OUT/parity.log"
B="timeout -k 10 200 python -u bench.py --no-cpu --steady-calls 8 --skip f64,f64_adaptive,config3,inter,config4,config5,extra,ab"
val() { python -c 'import json,sys; d=json.loads([l for l in sys.stdin if l.startswith("{")][-1]); a=d["adaptive"]; print(round(d["value"]/1e6,3), round(d["roofline"]["mean_launch_us"],1), round(d["steady_state"]["value"]/1e6,3), round(d["steady_state"]["kernel_us_per_call"],1), "ada", round(a["value"]/1e6,3), round(a["roofline"]["mean_launch_us"],1))'; }
for r in 1 2; do
  for v in splitbar splitbar2 nosplit; do
    for st in "20 5" "200 50"; do
      set -- $st
      echo "$v steps=$1 $(ODESAT_LIB=$PWD/expt/lib$v.so $B --steps $1 --warmup $2 2>/dev/null | val)" || exit 1
    done
  done
done
