#!/bin/bash
# Times the verify kernels of several builds (lachain_amd/ab/<tag>/liblachain_bls.so; "cur" = the in-tree build)
# on one small bench workload.  Usage: bash tools/ab_bench.sh OUTTAG tag1 tag2 ...
set -o pipefail
OUT=$1; shift
mkdir -p gpurun_out
for t in "$@"; do
  if [ "$t" = cur ]; then LIBP=""; else LIBP=$PWD/lachain_amd/ab/$t/liblachain_bls.so; fi
  LCB_LIB_PATH=$LIBP timeout -k 10 240 python -u bench.py --shares 262144 --steps 2 --warmup 1 --no-cpu-baseline \
      --ts-rounds ${TS_ROUNDS:-4096} --msm-sizes "${MSM_SIZES:-}" --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 > gpurun_out/${OUT}_$t.txt 2>&1 || { echo "$t FAILED"; tail -5 gpurun_out/${OUT}_$t.txt; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${OUT}_$t.txt').read().strip().splitlines()[-1])
r=d['roofline']; t=d['threshold_signature']
print('$t', 'tpke', round(d['value']), 'miller', round(r['kernel_ms']['k_tpke_miller'],2), 'fe', round(r['kernel_ms']['k_final_exp_check'],2), 'mism', d['config']['decision_mismatches'], '| ts', round(t['value']), round(t['phase_ms']['verify_shares'],2), t['decision_mismatches'])"
done
