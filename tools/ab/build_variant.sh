#!/bin/bash
# Build liblachain_bls.so with extra compile definitions into lachain_amd/ab/<tag>/ (A/B timing of kernel variants).
# Usage: bash tools/build_variant.sh TAG "-DFLAG1 -DFLAG2"
set -e
TAG=$1; DEFS=$2
R=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$R/build/ab_obj/$TAG
mkdir -p $OBJ $R/lachain_amd/ab/$TAG
make -s -j8 -C $R/lachain_amd/csrc OBJDIR=$OBJ OUT=$R/lachain_amd/ab/$TAG/liblachain_bls.so DEFS="$DEFS"
echo built $R/lachain_amd/ab/$TAG/liblachain_bls.so
