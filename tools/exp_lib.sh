#!/bin/bash
# Experiment build of the engine library: exp/libntc_gf256_<name>.so with extra compiler flags
# (A/B runs select it with NTC_GF256_LIB).  usage: bash tools/exp_lib.sh <name> [flags...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p $R/exp
C=$R/netcode_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -structurizecfg-skip-uniform-regions \
  -Wall -I $R/include "$@" -o $R/exp/libntc_gf256_$NAME.so $C/ntc_gf256.hip $C/ntc_dense.hip $C/ntc_wire.hip $C/ntc_gfw.hip
echo built exp/libntc_gf256_$NAME.so
