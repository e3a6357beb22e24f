#!/bin/bash
# exact TPKE this build vs lachain_amd/abfe, twice each, then the SQ stall counters (tools/gpu_pmc_ml.sh)
set -o pipefail
TAG=${1:-ml3}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
Z="--pattern-steps 0 --mcl-reps 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --ts-rounds 0 --tpke-batched 0 --headline exact --steps 3 --warmup 1"
OLD=lachain_amd/abfe/liblachain_bls.so
for rep in 1 2; do
  timeout -k 10 300 python3 -u bench.py $Z > gpurun_out/$TAG/new_$rep.txt 2>/dev/null || { echo new failed; exit 1; }
  LCB_LIB_PATH=$OLD timeout -k 10 300 python3 -u bench.py $Z > gpurun_out/$TAG/old_$rep.txt 2>/dev/null || { echo old failed; exit 1; }
  for v in new old; do python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/${v}_$rep.txt').read().strip().splitlines()[-1]); print('$v', '%.4g' % d['value'], '%.2f' % d['ms_per_step'], d['config']['decision_mismatches'])"; done
done
bash tools/gpu_pmc_ml.sh ${TAG}_pmc
