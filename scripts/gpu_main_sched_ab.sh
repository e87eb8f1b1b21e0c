#!/bin/bash
# The main translation unit (k_resident, k_wave, k_solo, k_step) built with the max-ILP machine
# scheduler (expt/libmainilp.so) against the product: the bench legs of those kernels and the
# criterion benches, alternated on one box.
set -u
o=gpurun_out/${TAG:-main_sched}; mkdir -p $o
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --only f64,f64_adaptive,config3,config4"
for r in 1 2; do
  for v in prod mainilp; do
    L=""; [ $v = mainilp ] && L=$PWD/expt/libmainilp.so
    ODESAT_LIB=$L $B > $o/$v.$r.log 2>&1 || exit 1
    ODESAT_LIB=$L timeout -k 10 120 python scripts/bench_criterion.py --no-cpu --calls 5 | sed "s/^/$v.$r /" >> $o/criterion.txt || exit 1
  done
done
python - <<'PY'
import json,glob,os
o=os.environ.get("TAG","main_sched")
for f in sorted(glob.glob(f"gpurun_out/{o}/*.[12].log")):
    d=[json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], *[(k, round(d[k]["value"]/1e6,3)) for k in ("f64","f64_adaptive","config3","inter_config4")])
PY
cat $o/criterion.txt
