#!/bin/bash
# TPKE batches in flight: 3 vs 4 (and 2), twice each, on this build
set -o pipefail
TAG=${1:-abpipe}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
B="--tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --steps 24 --warmup 2"
for rep in 1 2; do
  for P in 3 4 2; do
    timeout -k 10 300 python3 -u bench.py $B --tpke-pipeline $P > gpurun_out/$TAG/p${P}_$rep.txt 2> gpurun_out/$TAG/p${P}_$rep.err || { echo "P$P FAILED"; tail -5 gpurun_out/$TAG/p${P}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/p${P}_$rep.txt').read().strip().splitlines()[-1]); print('P$P', 'value %.4g' % d['value'], 'ms %.2f' % d['ms_per_step'], 'mism', d['config']['decision_mismatches'])"
  done
done
