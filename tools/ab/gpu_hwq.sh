#!/bin/bash
# batched TPKE, three in flight, at 6 / 8 / 12 hardware queues (bench --hw-queues), twice each
set -o pipefail
TAG=${1:-hwq}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
X="--pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --tpke-exact 0 --steps 21 --warmup 2"
for rep in 1 2; do
  for q in 6 8 12; do
    timeout -k 10 300 python3 -u bench.py $X --hw-queues $q > gpurun_out/$TAG/q${q}_$rep.txt 2>/dev/null || { echo "q$q failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/q${q}_$rep.txt').read().strip().splitlines()[-1]); print('q$q', '%.4g' % d['value'], '%.2f' % d['ms_per_step'], d['config']['decision_mismatches'])"
  done
done
