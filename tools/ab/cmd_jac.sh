#!/bin/bash
# Legendre symbols by the binary routine (base) vs the exponent (abv/jac0): GPU suite, then the headline and the
# preparation-bound / CommonCoin legs interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/jac
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/jac/gpu_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/jac/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/jac/gpu_tests.txt
T="--ts-rounds 65536 --ts-exact 0 --shares 4096 --tpke-pipeline 1"
bash tools/ab_tpke.sh jac "base:" "jac0:" "base:" "jac0:" "base:" "jac0:" "base:$T" "jac0:$T" "base:$T" "jac0:$T"
