#!/bin/bash
# Build an experimental variant of libodesat_hip.so with extra flags for onchip.hip:
#   scripts/build_variant.sh NAME "-DONCHIP_ORDER=1"   ->  expt/libNAME.so
# Run it with ODESAT_LIB=$PWD/expt/libNAME.so (scripts/expt.sh).  The product build is untouched.
set -eu
cd "$(dirname "$0")/.."
name=$1; flags=$2
mkdir -p build/vobj/$name expt
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wall -Wno-unused-function"
$H -fno-slp-vectorize $flags -c -o build/vobj/$name/onchip.o odesat_amd/csrc/onchip.hip
$H --offload-arch=gfx950 -shared -fPIC -o expt/lib$name.so build/vobj/$name/onchip.o build/obj/odesat_hip.o \
   build/obj/partition.o build/obj/cnf.o build/obj/preprocess.o build/obj/stoch.o
