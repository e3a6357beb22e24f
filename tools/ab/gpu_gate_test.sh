#!/bin/bash
# the scratch-gate GPU tests (concurrent assemblies) on this build, once
set -o pipefail
TAG=${1:-gate}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scratch_gate.py > gpurun_out/$TAG/tests.txt 2>&1 || { echo "TESTS FAILED"; grep -n "assert\|Error\|FAILED" gpurun_out/$TAG/tests.txt | head -20; exit 1; }
tail -3 gpurun_out/$TAG/tests.txt
