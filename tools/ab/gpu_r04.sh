#!/bin/bash
# Round-4 GPU call: the GPU suite, smoke, then the driver's bench command.  Usage: bash tools/gpu_r04.sh TAG
set -o pipefail
TAG=${1:-r04}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -X faulthandler -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.txt 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
  tail -c 3000 gpurun_out/${TAG}_bench.txt
fi
