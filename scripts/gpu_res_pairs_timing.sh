set -u
o=gpurun_out/r04ad; mkdir -p $o
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --only f64,f64_adaptive"
for r in 1 2; do
  $B > $o/prod.$r.log 2>&1 || exit 1
  ODESAT_LIB=$PWD/expt/libpairs.so $B > $o/pairs.$r.log 2>&1 || exit 1
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r04ad/*.[12].log")):
    d=[json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], *[(k, round(d[k]["value"]/1e6,3), round(d[k]["roofline"]["mean_launch_us"],1)) for k in ("f64","f64_adaptive")])
PY
