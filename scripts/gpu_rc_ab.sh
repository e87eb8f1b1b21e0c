#!/bin/bash
# f64 fixed k_resident with register-cached tiles (resident.hpp, RES_RC): parity first, then the
# bench's f64 leg alternated -- product (RES_RC=28), ODESAT_RES_RC=0 (all tiles stream), rc20.
set -u
o=gpurun_out/${TAG:-rc_ab}; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "${TESTK:-f64 or resident or fuzz}" > $o/pytest.log 2>&1; rc=$?; tail -2 $o/pytest.log; [ $rc = 0 ] || exit 1
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --only f64"
for r in 1 2; do
  $B > $o/prod.$r.log 2>&1 || exit 1
  ODESAT_RES_RC=0 $B > $o/off.$r.log 2>&1 || exit 1
  ODESAT_LIB=$PWD/expt/librc20.so $B > $o/rc20.$r.log 2>&1 || exit 1
done
python - <<'PY'
import json,glob,os
o=os.environ.get("TAG","rc_ab")
for f in sorted(glob.glob(f"gpurun_out/{o}/*.[12].log")):
    d=[json.loads(l) for l in open(f) if l.startswith("{")][-1]
    x=d["f64"]; print(f.split("/")[-1], round(x["value"]/1e6,3), round(x["ms_per_step"]*1e3,1), round(x["roofline"]["mean_launch_us"],1), x["kernel"])
PY
