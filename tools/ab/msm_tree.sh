#!/bin/bash
# MSM / mcl GPU tests, then the 2^20 MSM one at a time (10 steps): cooperative tree (base) vs serial tree (abv/tree0)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/msmtree
timeout -k 10 600 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_multirank.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/msmtree/gpu_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/msmtree/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/msmtree/gpu_tests.txt
X="--shares 22528 --steps 1 --warmup 1 --tpke-pipeline 1 --tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --msm-sizes 1048576 --msm-steps 10"
for i in 1 2 3 4 5 6; do
  if (( i % 2 )); then unset LCB_LIB_PATH; tag=coop; else export LCB_LIB_PATH=$R/lachain_amd/abv/tree0/liblachain_bls.so; tag=serial; fi
  timeout -k 10 300 python -u bench.py $X > gpurun_out/msmtree/b$i.txt 2> gpurun_out/msmtree/b$i.err || { echo "BENCH FAILED"; tail -5 gpurun_out/msmtree/b$i.err; exit 1; }
  echo "$tag $(grep -o '"single_msm": {[^}]*}' gpurun_out/msmtree/b$i.txt | head -1) $(grep -o '"phase_ms": {"digits[^}]*}' gpurun_out/msmtree/b$i.txt | head -1)"
done
