#!/bin/bash
# A/B at three (and four) batches in flight: this build vs the previous commit's (lachain_amd/abfe), level-1 Miller
# loop on the one-lane kernel (coop-miller-max 32768), four batches in flight.  Usage: bash tools/gpu_ab2.sh TAG
set -o pipefail
TAG=${1:-ab2}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
X="--pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --tpke-exact 0 --steps 21 --warmup 2"
run() {
  name=$1; shift
  "$@" > gpurun_out/$TAG/$name.txt 2> gpurun_out/$TAG/$name.err || { echo "$name FAILED"; tail -20 gpurun_out/$TAG/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/$name.txt').read().strip().splitlines()[-1]); print('$name', 'value %.4g' % d['value'], 'ms %.2f' % d['ms_per_step'], 'mism', d['config'].get('decision_mismatches'))"
}
OLD=lachain_amd/abfe/liblachain_bls.so
for rep in 1 2; do
  run new_$rep timeout -k 10 300 python3 -u bench.py $X
  run old_$rep env LCB_LIB_PATH=$OLD timeout -k 10 300 python3 -u bench.py $X
  run ml32k_$rep env LCB_ALLOW_TUNING=1 timeout -k 10 300 python3 -u bench.py $X --coop-miller-max 32768
done
run p4 timeout -k 10 300 python3 -u bench.py $X --tpke-pipeline 4
run p4q16 timeout -k 10 300 python3 -u bench.py $X --tpke-pipeline 4 --hw-queues 16
run exact timeout -k 10 300 python3 -u bench.py --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --tpke-batched 0 --headline exact --steps 3 --warmup 1
