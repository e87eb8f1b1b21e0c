# A/B of k_solo builds on the criterion benches (same box, alternated): expt/libsoloold.so vs the tree.
set -u
mkdir -p gpurun_out
: > gpurun_out/solo_ab.txt
for rep in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export ODESAT_LIB=$PWD/expt/libsoloold.so; else unset ODESAT_LIB; fi
    echo "== $v" >> gpurun_out/solo_ab.txt
    timeout -k 10 120 python -u scripts/bench_criterion.py --no-cpu --calls 10 2>/dev/null >> gpurun_out/solo_ab.txt || { echo "crit $v failed"; exit 1; }
  done
done
cat gpurun_out/solo_ab.txt
