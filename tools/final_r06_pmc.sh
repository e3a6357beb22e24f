#!/bin/bash
# Round-6 evidence, part 2 (one GPU call): PMC passes of the exact TPKE pair (262,144 shares) and of one batched step,
# folded ON THE BOX into profiles/pmc_tpke_*.json (so the bench that follows attaches this build's traffic), then the
# driver's bench command.  Usage: bash tools/final_r06_pmc.sh TAG
set -o pipefail
TAG=${1:-r06p}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
PMC_CMD="python3 $R/bench.py --shares 262144 --steps 1 --warmup 0 --no-cpu-baseline --tpke-batched 0 --headline exact --pattern-steps 0 --mcl-reps 0 --ts-batched 0 --ts-rounds 4096 --msm-steps 1 --msm-sizes 1048576 --msm-pipeline 1 --replay-n 0 --ecdsa-sigs 262144 --ecdsa-steps 1 --dkg-n 0 --rs-n 0" bash tools/pmc_round.sh ${TAG}_exact || exit 1
PMC_CMD="python3 $R/bench.py --tpke-exact 0 --tpke-pipeline 1 --steps 1 --warmup 0 --no-cpu-baseline --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0" bash tools/pmc_round.sh ${TAG}_batched || exit 1
python3 tools/pmc_to_json.py profiles/pmc_tpke_verify.json 262144 1048576 gpurun_out/pmc_${TAG}_exact_{1,2,3}/run_counter_collection.csv || exit 1
python3 tools/pmc_batched_to_json.py profiles/pmc_tpke_batched.json gpurun_out/pmc_${TAG}_batched_{1,2,3}/run_counter_collection.csv || exit 1
mkdir -p gpurun_out/$TAG/pmc && cp profiles/pmc_tpke_verify.json profiles/pmc_tpke_batched.json gpurun_out/$TAG/pmc/
echo pmc done
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench_full.txt 2> gpurun_out/$TAG/bench_progress.txt || { echo "BENCH FAILED"; tail -20 gpurun_out/$TAG/bench_progress.txt; exit 1; }
tail -c 1200 gpurun_out/$TAG/bench_full.txt
