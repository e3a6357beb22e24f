#!/bin/bash
# A/B on the final build: three or four TPKE batches in flight (bench.py --tpke-pipeline), interleaved, three reps
set -o pipefail
TAG=${1:-abpipe4}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
B="--tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --steps 20 --warmup 5"
run() {
  name=$1; shift
  "$@" > gpurun_out/$TAG/$name.txt 2> gpurun_out/$TAG/$name.err || { echo "$name FAILED"; tail -20 gpurun_out/$TAG/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/$name.txt').read().strip().splitlines()[-1]); print('$name', 'value %.4g' % d['value'], 'ms %.2f' % d['ms_per_step'], 'mism', d['config']['decision_mismatches'])"
}
for rep in 1 2 3; do
run p3_$rep timeout -k 10 300 python3 -u bench.py $B --tpke-pipeline 3
run p4_$rep timeout -k 10 300 python3 -u bench.py $B --tpke-pipeline 4
done
echo done
