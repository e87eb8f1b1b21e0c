set -e
o=gpurun_out/r04t; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "call_sequences" > $o/pytest.log 2>&1
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --only none > $o/plain$i.log 2>&1
  ODESAT_BENCH_DIST=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --only none > $o/dist$i.log 2>&1
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r04t/*.log")):
    if "pytest" in f: print(f, open(f).read().strip().splitlines()[-1]); continue
    d=[json.loads(l) for l in open(f) if l.startswith("{")][-1]
    r=d["roofline"]; print(f, round(d["value"]/1e6,3), round(d["ms_per_step"]*20e3,1), round(r["mean_launch_us"],1), round(d["steady_state"]["value"]/1e6,3))
PY
