#!/bin/bash
# Round-end evidence in ONE GPU call: the GPU suite, smoke, rocprofv3 kernel trace of the bench, the PMC passes
# folded into profiles/pmc_tpke_*.json ON THE BOX (so the driver-command bench that follows attaches the traffic of
# this very build), then the driver's bench command.  Outputs under gpurun_out/<TAG>_*.  Usage: bash tools/final_all.sh TAG
set -o pipefail
TAG=${1:-final}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -X faulthandler -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
bash tools/final_round.sh ${TAG} || exit 1
cd $R
python3 tools/pmc_to_json.py profiles/pmc_tpke_verify.json 262144 1048576 gpurun_out/pmc_${TAG}_exact_{1,2,3}/run_counter_collection.csv || exit 1
python3 tools/pmc_batched_to_json.py profiles/pmc_tpke_batched.json gpurun_out/pmc_${TAG}_batched_{1,2,3}/run_counter_collection.csv || exit 1
mkdir -p gpurun_out/${TAG}_pmc && cp profiles/pmc_tpke_verify.json profiles/pmc_tpke_batched.json gpurun_out/${TAG}_pmc/
timeout -k 10 700 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.txt 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
tail -c 1500 gpurun_out/${TAG}_bench.txt
