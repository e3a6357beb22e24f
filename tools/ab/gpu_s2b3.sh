#!/bin/bash
# VERDICT r4 #2, third step: the failing open-list-position build against the same build with IPRA off
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && rm -rf gpurun_out/s2b && mkdir -p gpurun_out/s2b
export LCB_ALLOW_TEST_HOOKS=1 LCB_ALLOW_FIXED_BATCH_SEED=1 LCB_ALLOW_TUNING=1 S2B_ITERS=1
for v in s2pos s2pos_noipra; do
  LCB_LIB_PATH=$R/lachain_amd/ab/$v/liblachain_bls.so timeout -k 10 200 python -u tools/debug/search2b_ab.py run $v 64 > gpurun_out/s2b/run_$v.txt 2>&1 || { echo "$v RUN FAILED"; tail -20 gpurun_out/s2b/run_$v.txt; exit 1; }
  grep '^{' gpurun_out/s2b/run_$v.txt
done
rm -f gpurun_out/s2b/*.bin
