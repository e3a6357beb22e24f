#!/bin/bash
# MSM-only bench (configs[3]) for each record chunk size K in $KS (LCB_MSM_CHUNK), 5 steps per size.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for K in ${KS:-64 32 128}; do
  LCB_ALLOW_TUNING=1 LCB_MSM_CHUNK=$K timeout -k 10 300 python3 -u bench.py --tpke-exact 1 --tpke-batched 0 --headline exact --ts-rounds 0 --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --mcl-reps 0 --no-cpu-baseline --pattern-steps 0 --shares 22000 --steps 1 --warmup 1 --msm-steps 5 > gpurun_out/msmab_$K.txt 2> gpurun_out/msmab_$K.err || { echo "BENCH FAILED K=$K"; tail -5 gpurun_out/msmab_$K.err; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/msmab_$K.txt') if l.startswith('BENCH_DETAIL')][-1][13:])
for m in d['msm']: print('K=$K', m['total_points'], round(m['value'] / 1e6, 1), 'M/s', round(m['ms_per_step'], 3), m['phase_ms'], m['known_answer_ok'])"
done
