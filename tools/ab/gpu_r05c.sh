#!/bin/bash
# MSM with 1/2/3 in flight, then a rocprofv3 kernel trace of the TPKE batched bench with three batches in flight
# (occupancy / overlap: tools/pipe_profile.py).  Usage: bash tools/gpu_r05c.sh TAG
set -o pipefail
TAG=${1:-r05c}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
bash tools/gpu_msm.sh $TAG || exit 1
B="--tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/prof -o run -- python3 $R/bench.py $B --tpke-pipeline 3 --steps 9 --warmup 2 > $R/gpurun_out/$TAG/bench_rocprof.txt 2>&1 || { echo "ROCPROF FAILED"; tail -5 $R/gpurun_out/$TAG/bench_rocprof.txt; exit 1; }
cd $R && gzip -f gpurun_out/$TAG/prof/run_kernel_trace.csv && ls -la gpurun_out/$TAG/prof && echo done
