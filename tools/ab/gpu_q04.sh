#!/bin/bash
# Round-4 quick GPU call: selected GPU tests (TESTS), then TPKE-only bench lines for each pipeline depth in PIPES, then
# (MCL=1) the mcl latency section.  Usage: TESTS="tests/test_gpu_ptmul.py" PIPES="1 2" bash tools/gpu_q04.sh TAG
set -o pipefail
TAG=${1:-q}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -X faulthandler -m pytest $TESTS -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
  tail -2 gpurun_out/${TAG}_tests.txt
fi
for HQ in ${HWQS:-0}; do
for PR in ${PRIOS:-1}; do
for P in $PIPES; do
  LCB_BENCH_HWQ=$HQ LCB_ALLOW_TUNING=1 LCB_WAVE_PRIO=$PR timeout -k 10 300 python3 -u bench.py --tpke-exact 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --mcl-reps 0 --no-cpu-baseline --pattern-steps 0 --steps ${STEPS:-10} --warmup 2 --tpke-pipeline $P > gpurun_out/${TAG}_p${P}_w${PR}_q$HQ.txt 2> gpurun_out/${TAG}_p${P}_w${PR}_q$HQ.err || { echo "BENCH FAILED p$P"; tail -20 gpurun_out/${TAG}_p${P}_w${PR}_q$HQ.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_p${P}_w${PR}_q$HQ.txt').read().strip().splitlines()[-1]); s=d.get('tpke_single_batch') or {}; print('hwq $HQ prio $PR pipe $P', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],2), 'ms', d['config']['decision_mismatches'], 'mism; single', s.get('value'), s.get('ms_per_step'))"
done
done
done
if [ -n "$MSMB" ]; then
  for SG in ${MSMSEGS:-0}; do
  for K in $MSMB; do
    LCB_MSM_SEGS=$SG LCB_ALLOW_TUNING=1 LCB_MSM_CHUNK=$K timeout -k 10 300 python3 -u bench.py --tpke-exact 0 --tpke-batched 0 --ts-rounds 0 --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --mcl-reps 0 --no-cpu-baseline --pattern-steps 0 --shares 22000 --headline exact --tpke-exact 1 --steps 1 --warmup 1 --msm-steps 5 > gpurun_out/${TAG}_msm$K.txt 2> gpurun_out/${TAG}_msm$K.err || { echo "MSM BENCH FAILED"; tail -20 gpurun_out/${TAG}_msm$K.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/${TAG}_msm$K.txt') if l.startswith('BENCH_DETAIL')][-1][13:]); [print('msm segs $SG chunk $K', m['total_points'], round(m['value']/1e6,1), 'M/s', m['ms_per_step'], m['phase_ms'], m['known_answer_ok']) for m in d['msm']]"
  done
  done
fi
if [ -n "$MCL" ]; then
  timeout -k 10 300 python3 -u bench.py --tpke-exact 0 --tpke-batched 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --mcl-reps 30 --no-cpu-baseline --pattern-steps 0 --shares 22000 --headline exact --tpke-exact 1 --steps 1 --warmup 1 > gpurun_out/${TAG}_mcl.txt 2> gpurun_out/${TAG}_mcl.err || { echo "MCL BENCH FAILED"; tail -20 gpurun_out/${TAG}_mcl.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_mcl.txt').read().strip().splitlines()[-1]); print(d['summary']['mcl_latency_us'])"
fi
