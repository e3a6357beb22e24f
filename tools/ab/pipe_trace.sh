#!/bin/bash
# Kernel trace of the pipelined TPKE headline alone (20 steps, three batches in flight) for the steady-state GPU-time split.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pipe
cd /tmp && export TMPDIR=/tmp
B="--steps 20 --warmup 5 --tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pipe/tr -o run -- python3 $R/bench.py $B > $R/gpurun_out/pipe/bench.txt 2>&1 || { echo FAILED; tail -5 $R/gpurun_out/pipe/bench.txt; exit 1; }
gzip -f $R/gpurun_out/pipe/tr/run_kernel_trace.csv
tail -c 300 $R/gpurun_out/pipe/bench.txt
