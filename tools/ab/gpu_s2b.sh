#!/bin/bash
# the two-error search's addressing variants side by side (stage dumps, tools/debug/search2b_ab.py), the
# batched GPU tests, then a TPKE-only bench at the driver's step count.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/s2b
export LCB_ALLOW_TEST_HOOKS=1 LCB_ALLOW_FIXED_BATCH_SEED=1 LCB_ALLOW_TUNING=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_batched.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s2b/tests.txt 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/s2b/tests.txt; exit 1; }
tail -2 gpurun_out/s2b/tests.txt
timeout -k 10 200 python -u tools/debug/search2b_ab.py run base > gpurun_out/s2b/run_base.txt 2>&1 || { echo "BASE RUN FAILED"; tail -20 gpurun_out/s2b/run_base.txt; exit 1; }
cat gpurun_out/s2b/run_base.txt | grep '^{'
LCB_LIB_PATH=$R/lachain_amd/ab/s2pos/liblachain_bls.so timeout -k 10 200 python -u tools/debug/search2b_ab.py run pos > gpurun_out/s2b/run_pos.txt 2>&1 || { echo "POS RUN FAILED"; tail -20 gpurun_out/s2b/run_pos.txt; exit 1; }
cat gpurun_out/s2b/run_pos.txt | grep '^{'
for c in 0 1 2; do python tools/debug/search2b_ab.py compare gpurun_out/s2b/base gpurun_out/s2b/pos $c || true; done
unset LCB_ALLOW_TEST_HOOKS LCB_ALLOW_FIXED_BATCH_SEED LCB_ALLOW_TUNING
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 --tpke-exact 0 --pattern-steps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --mcl-reps 0 --no-cpu-baseline > gpurun_out/s2b/bench.json 2> gpurun_out/s2b/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/s2b/bench.err; exit 1; }
tail -1 gpurun_out/s2b/bench.json | cut -c1-700
