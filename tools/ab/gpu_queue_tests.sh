#!/bin/bash
# the queue / cache GPU tests on this build
set -o pipefail
TAG=${1:-qtests}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_queue.py tests/test_gpu_ct_cache.py > gpurun_out/$TAG/tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$TAG/tests.txt; exit 1; }
tail -8 gpurun_out/$TAG/tests.txt
