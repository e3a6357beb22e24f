#!/bin/bash
# mcl hashAndMapTo with the cofactor clearing on four-lane groups (base) vs one lane (abv/mhc0): hash / mcl GPU tests,
# then the mcl single-call latencies of both builds, twice
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/mhc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sign_convention.py tests/test_gpu_mcl_surface.py tests/test_gpu_ts_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mhc/gpu_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/mhc/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/mhc/gpu_tests.txt
X="--shares 22528 --steps 1 --warmup 1 --tpke-pipeline 1 --tpke-exact 0 --pattern-steps 0 --mcl-reps 200 --ts-rounds 0 --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --msm-sizes="
for i in 1 2 3 4; do
  if (( i % 2 )); then unset LCB_LIB_PATH; tag=coop; else export LCB_LIB_PATH=$R/lachain_amd/abv/mhc0/liblachain_bls.so; tag=one_lane; fi
  timeout -k 10 400 python -u bench.py $X > gpurun_out/mhc/b$i.txt 2> gpurun_out/mhc/b$i.err || { echo "BENCH FAILED"; tail -5 gpurun_out/mhc/b$i.err; exit 1; }
  echo "$tag $(grep -o '"mcl_latency_us":{[^}]*}' gpurun_out/mhc/b$i.txt | head -1)"
done
