#!/bin/bash
# mclBnG1_mul on four 65-bit ladders with the membership test on the host: ptmul / mcl / configs GPU tests, then the
# mcl single-call latencies (twice)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/g1mul
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g1mul/gpu_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/g1mul/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/g1mul/gpu_tests.txt
X="--shares 22528 --steps 1 --warmup 1 --tpke-pipeline 1 --tpke-exact 0 --pattern-steps 0 --mcl-reps 300 --ts-rounds 0 --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --msm-sizes="
for i in 1 2; do
  timeout -k 10 400 python -u bench.py $X > gpurun_out/g1mul/b$i.txt 2> gpurun_out/g1mul/b$i.err || { echo "BENCH FAILED"; tail -5 gpurun_out/g1mul/b$i.err; exit 1; }
  grep -o '"mcl_latency_us":{[^}]*}' gpurun_out/g1mul/b$i.txt | head -1
done
