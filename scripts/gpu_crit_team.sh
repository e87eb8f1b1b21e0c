set -u
cd $GRAFT_REPO_ROOT
for t in auto 1 2 4; do
  if [ $t = auto ]; then unset ODESAT_WAVE_TEAM; else export ODESAT_WAVE_TEAM=$t; fi
  echo "team=$t"; timeout -k 10 300 python scripts/bench_criterion.py --calls 3 --no-cpu 2>&1 | tail -3
done
