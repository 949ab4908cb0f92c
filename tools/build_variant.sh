#!/bin/bash
# Build a variant of libntc_gf256.so for A/B runs (tools/ab_lib.sh / NTC_GF256_LIB=<path>).
# usage: bash tools/build_variant.sh <out.so> [<git rev>|-] [extra hipcc flags...]
#   <git rev>: build the csrc/ of that commit (from git show into a temp dir); "-": the working tree
set -e
OUT=$1; REV=${2:--}; shift 2 || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/netcode_amd/csrc
if [ "$REV" != "-" ]; then
  TMP=$(mktemp -d); mkdir -p $TMP/csrc
  for f in ntc_gf256.hip ntc_dense.hip ntc_wire.hip ntc_gfw.hip engine.hh gf256_field.hh gf_bitslice_table.inc; do
    git -C $ROOT show $REV:netcode_amd/csrc/$f > $TMP/csrc/$f
  done
  SRC=$TMP/csrc
fi
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -structurizecfg-skip-uniform-regions \
  -Wall -I $ROOT/include "$@" -o "$OUT" $SRC/ntc_gf256.hip $SRC/ntc_dense.hip $SRC/ntc_wire.hip $SRC/ntc_gfw.hip
echo "built $OUT"
