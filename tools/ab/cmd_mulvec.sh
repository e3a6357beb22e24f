#!/bin/bash
# GPU suite, then mcl single-call latencies with mulVec / G1 Lagrange on the cooperative ladders (base) vs the
# one-lane per-term kernels (LCB_MULVEC_COOP=0), interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/mulvec
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mulvec/gpu_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/mulvec/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/mulvec/gpu_tests.txt
X="--shares 22528 --steps 1 --warmup 1 --tpke-pipeline 1 --tpke-exact 0 --pattern-steps 0 --mcl-reps 200 --ts-rounds 0 --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --msm-sizes="
for i in 1 2 3 4; do
  if (( i % 2 )); then tag=coop; E=1; else tag=one_lane; E=0; fi
  LCB_MULVEC_COOP=$E timeout -k 10 400 python -u bench.py $X > gpurun_out/mulvec/b$i.txt 2> gpurun_out/mulvec/b$i.err || { echo "BENCH FAILED"; tail -5 gpurun_out/mulvec/b$i.err; exit 1; }
  echo "$tag $(grep -o '"mcl_latency_us":{[^}]*}' gpurun_out/mulvec/b$i.txt | head -1)"
done
