#!/bin/bash
# A/B of the batched step's kernel forms with three batches in flight: level-1 Miller loop / final exponentiation on
# the nine-lane (coop) or one-lane kernels, and the latency kernels' wave priority.  Usage: bash tools/gpu_ab_coop.sh TAG
set -o pipefail
TAG=${1:-abcoop}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
B="--tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --steps 21 --warmup 2 --tpke-pipeline ${P:-3}"
run() {
  name=$1; shift
  env LCB_ALLOW_TUNING=1 "$@" > gpurun_out/$TAG/$name.txt 2> gpurun_out/$TAG/$name.err || { echo "$name FAILED"; tail -20 gpurun_out/$TAG/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/$name.txt').read().strip().splitlines()[-1]); print('$name', 'value %.4g' % d['value'], 'ms %.2f' % d['ms_per_step'], 'mism', d['config']['decision_mismatches'])"
}
run base timeout -k 10 300 python3 -u bench.py $B
run ml32k timeout -k 10 300 python3 -u bench.py $B --coop-miller-max 32768
run co64k timeout -k 10 300 python3 -u bench.py $B --coop-max 65536
run co0 timeout -k 10 300 python3 -u bench.py $B --coop-max 0
run prio0 env LCB_WAVE_PRIO=0 timeout -k 10 300 python3 -u bench.py $B
