#!/bin/bash
# Build an experimental variant of libodesat_hip.so: SRC (default onchip) is recompiled with extra
# flags from the working tree, every other object comes from the product build (make first):
#   scripts/build_variant.sh NAME "-DFLAG" [SRC]   ->  expt/libNAME.so
# Run it with XP_LIB=$PWD/expt/libNAME.so (scripts/tooling.py; bench.py --lib; scripts/gpu_ab.sh).
set -eu
cd "$(dirname "$0")/.."
name=$1; flags=$2; src=${3:-onchip}
mkdir -p build/vobj/$name expt
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wall -Wno-unused-function"
extra=""; [ "$src" = onchip ] && extra="-fno-slp-vectorize -mllvm -amdgpu-sched-strategy=max-ilp"  # (the Makefile's ONCHIP_FLAGS)
[ "$src" = wave_k ] && extra="-mllvm -amdgpu-sched-strategy=max-ilp"  # (WAVE_FLAGS)
$H $extra $flags -c -o build/vobj/$name/$src.o odesat_amd/csrc/$src.hip
objs=""
for o in odesat_hip onchip wave_k partition cnf preprocess stoch run_abi experiment cv_layout; do
  if [ "$o" = "$src" ]; then objs="$objs build/vobj/$name/$o.o"; else objs="$objs build/obj/$o.o"; fi
done
$H -shared -fPIC -o expt/lib$name.so $objs
