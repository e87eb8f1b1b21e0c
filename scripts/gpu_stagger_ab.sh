# A/B: k_onchip's first round of workgroups started in four phases (ODESAT_ONCHIP_STAGGER_TICKS,
# 100 MHz ticks per phase) on the driver-shaped headline (20 steps) and the 200-step line.
set -u
B="timeout -k 10 120 python bench.py --no-cpu --skip f64,adaptive,inter,config4,config5,extra,ab"
val() { python -c 'import json,sys; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][0]); print(round(d["value"]), round(d["roofline"]["mean_launch_us"],1))'; }
for r in 1 2; do
  for t in 0 200 400 800 1500; do
    for st in "20 5" "200 50"; do
      set -- $st
      echo "ticks=$t steps=$1 $(ODESAT_ONCHIP_STAGGER_TICKS=$t $B --steps $1 --warmup $2 | val)" || exit 1
    done
  done
done
