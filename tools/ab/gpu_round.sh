#!/bin/bash
# One GPU round: parity tests, bench, rocprofv3 kernel stats (csv).  Usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -3 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.txt 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/${TAG}_bench.txt; exit 1; }
tail -1 gpurun_out/${TAG}_bench.txt
if [ -n "$PROF" ]; then
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --no-cpu-baseline --replay-n 0 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_bench_rocprof.txt 2>&1) || { echo "ROCPROF FAILED"; exit 1; }
  find gpurun_out/prof_${TAG} -name "*stats*"
fi
