#!/bin/bash
# Build liblachain_bls.so with extra compile definitions into lachain_amd/abv/<tag>/ (A/B timing of kernel variants;
# git-ignored, not gpurun-ignored, so it travels to the GPU box; select it with LCB_LIB_PATH).
# Usage: bash tools/build_variant.sh TAG "-DFLAG1 -DFLAG2"
set -e
TAG=$1; DEFS=$2
R=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$R/build/ab_obj/$TAG
mkdir -p $OBJ $R/lachain_amd/abv/$TAG
make -s -j8 -C $R/lachain_amd/csrc OBJDIR=$OBJ OUT=$R/lachain_amd/abv/$TAG/liblachain_bls.so DEFS="$DEFS"
echo built $R/lachain_amd/abv/$TAG/liblachain_bls.so
