# A/B of adaptive k_onchip: product vs expt/lib$VAR.so on the bench's adaptive leg (20 and 200
# steps, alternated), then the variant's adaptive parity tests.
set -u
B="timeout -k 10 120 python bench.py --no-cpu --only adaptive"
val() { python -c 'import json,sys; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][0]); a=d["adaptive"]; print(round(a["value"]), round(a["roofline"]["mean_launch_us"],1))'; }
for r in 1 2; do
  for st in "20 5" "200 20"; do
    set -- $st
    echo "prod steps=$1 $($B --steps $1 --warmup $2 | val)" || exit 1
    echo "$VAR steps=$1 $(ODESAT_LIB=$PWD/expt/lib$VAR.so $B --steps $1 --warmup $2 | val)" || exit 1
  done
done
ODESAT_LIB=$PWD/expt/lib$VAR.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "onchip or algorithms_identical" 2>&1 | tail -2
