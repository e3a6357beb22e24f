#!/bin/bash
# A/B with three TPKE batches in flight: the level checks' nine-lane final exponentiation at 284 registers (k_coop.hip)
# or 248 (the k_prep.hip copy, LCB_COOP_FE_2W=1), with level 1 on the one-lane kernel (default) or the nine-lane one
set -o pipefail
TAG=${1:-abfe2w}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
B="--tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --steps 21 --warmup 2 --tpke-pipeline 3"
run() {
  name=$1; shift
  env LCB_ALLOW_TUNING=1 "$@" > gpurun_out/$TAG/$name.txt 2> gpurun_out/$TAG/$name.err || { echo "$name FAILED"; tail -20 gpurun_out/$TAG/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/$name.txt').read().strip().splitlines()[-1]); print('$name', 'value %.4g' % d['value'], 'ms %.2f' % d['ms_per_step'], 'mism', d['config']['decision_mismatches'])"
}
for rep in 1 2; do
run base$rep timeout -k 10 300 python3 -u bench.py $B
run fe2w$rep env LCB_COOP_FE_2W=1 timeout -k 10 300 python3 -u bench.py $B
run fe2w_co64k$rep env LCB_COOP_FE_2W=1 timeout -k 10 300 python3 -u bench.py $B --coop-max 65536
done
