#!/bin/bash
# the aggregation queue on this build: its GPU tests, the queue bench (16 / 64 one-share callers), and a kernel trace
# at 64 callers (1 ms deadline): what a flush's chain is made of
set -o pipefail
TAG=${1:-qprof}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_queue.py tests/test_gpu_ct_cache.py > gpurun_out/$TAG/tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$TAG/tests.txt; exit 1; }
tail -3 gpurun_out/$TAG/tests.txt
timeout -k 10 300 python3 -u tools/queue_bench.py --seconds 3 --deadlines 0,1,5 > gpurun_out/$TAG/queue_bench.jsonl 2> gpurun_out/$TAG/queue_bench.err || { echo "QUEUE BENCH FAILED"; tail -5 gpurun_out/$TAG/queue_bench.err; exit 1; }
cat gpurun_out/$TAG/queue_bench.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/rocprof -o run -- python3 $R/tools/queue_bench.py --seconds 2 --deadlines 1 --threads 64 > $R/gpurun_out/$TAG/queue_prof.txt 2>&1 || { echo "PROF FAILED"; tail -5 $R/gpurun_out/$TAG/queue_prof.txt; exit 1; }
tail -2 $R/gpurun_out/$TAG/queue_prof.txt
