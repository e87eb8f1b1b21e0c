#!/bin/bash
# f64 adaptive k_resident (VFG) with register tiles (RES_RC_ADA): parity, then the bench's
# f64_adaptive and f64 legs, product vs ODESAT_RES_RC=0, alternated.
set -u
o=gpurun_out/${TAG:-rca_ab}; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "${TESTK:-f64 or resident or fuzz or register}" > $o/pytest.log 2>&1; rc=$?; tail -2 $o/pytest.log; [ $rc = 0 ] || exit 1
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --only f64,f64_adaptive"
for r in 1 2; do
  $B > $o/prod.$r.log 2>&1 || exit 1
  ODESAT_RES_RC=0 $B > $o/off.$r.log 2>&1 || exit 1
done
python - <<'PY'
import json,glob,os
o=os.environ.get("TAG","rca_ab")
for f in sorted(glob.glob(f"gpurun_out/{o}/*.[12].log")):
    d=[json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], *[(k, round(d[k]["value"]/1e6,3), round(d[k]["roofline"]["mean_launch_us"],1)) for k in ("f64","f64_adaptive")])
PY
