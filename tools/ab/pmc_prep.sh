#!/bin/bash
# GPU tests, then FETCH_SIZE / WRITE_SIZE passes of one batched TPKE step in fork mode 4 (one preparation dispatch) and
# fork mode 3 (hash and point lanes as separate kernels), folded per kernel.  Usage: bash tools/ab/pmc_prep.sh TAG
set -o pipefail
TAG=${1:-pp}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/$TAG/gpu_tests.txt 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/$TAG/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/$TAG/gpu_tests.txt
for fm in 4 3; do
  PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" PMC_CMD="python3 $R/bench.py --tpke-exact 0 --tpke-pipeline 1 --steps 1 --warmup 0 --no-cpu-baseline --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --fork-mode $fm" bash tools/pmc_round.sh ${TAG}_fm$fm || exit 1
  python3 tools/pmc_batched_to_json.py gpurun_out/$TAG/fm$fm.json gpurun_out/pmc_${TAG}_fm${fm}_{1,2}/run_counter_collection.csv || exit 1
done
echo done
