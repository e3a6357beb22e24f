#!/bin/bash
# Quick GPU iteration: selected GPU tests (TESTS, pytest -k expression or file list) then a TPKE-only bench with rocprof
# kernel trace.  Usage: TESTS="tests/test_gpu_batched.py" bash tools/gpu_quick.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-q}; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
  tail -2 gpurun_out/${TAG}_tests.txt
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --tpke-exact 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --mcl-reps 0 --no-cpu-baseline "$@" > $R/gpurun_out/${TAG}_bench.json 2> $R/gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 $R/gpurun_out/${TAG}_bench.err; exit 1; }
cd $R && python3 tools/trace_by_grid.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/${TAG}_grid.txt && head -40 gpurun_out/${TAG}_grid.txt
if [ -n "$QUEUE" ]; then
  timeout -k 10 300 python3 -u tools/queue_bench.py $QUEUE > gpurun_out/${TAG}_queue.jsonl 2> gpurun_out/${TAG}_queue.err || { echo "QUEUE FAILED"; tail -20 gpurun_out/${TAG}_queue.err; exit 1; }
  cat gpurun_out/${TAG}_queue.jsonl
fi
