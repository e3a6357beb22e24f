#!/bin/bash
# MSM configs[3] with 1, 2 and 3 independent MSMs in flight (bench.py --msm-pipeline)
set -o pipefail
TAG=${1:-msm}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
B="--shares 22528 --steps 1 --tpke-pipeline 1 --tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline"
for P in ${PIPES:-1 2 3}; do
  timeout -k 10 300 python3 -u bench.py $B --msm-steps 4 --warmup 1 --msm-pipeline $P > gpurun_out/$TAG/msm_p$P.txt 2> gpurun_out/$TAG/msm_p$P.err || { echo "MSM BENCH FAILED"; tail -20 gpurun_out/$TAG/msm_p$P.err; exit 1; }
  python3 - $TAG $P <<'PY'
import json, sys, glob, os
tag, p = sys.argv[1], sys.argv[2]
f = max(glob.glob('gpurun_out/bench_detail_*.json'), key=os.path.getmtime)
for m in json.load(open(f))['msm']:
    print('P', p, m['total_points'], 'value %.4g' % m['value'], 'ms %.3f' % m['ms_per_step'], 'single %.3f' % m['single_msm']['ms'],
          'ok', m['known_answer_ok'], 'frac_acc %.3f' % m['roofline']['frac'], 'frac_whole %.3f' % m['frac_whole_msm'])
PY
done
