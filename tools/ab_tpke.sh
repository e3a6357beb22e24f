#!/bin/bash
# A/B of the TPKE headline (no other bench legs): each argument is "LIBTAG:bench flags", LIBTAG "base" for the
# in-tree library or a tools/build_variant.sh tag (lachain_amd/abv/TAG).  One summary line per run.
# Usage: bash tools/ab_tpke.sh OUT_TAG "base:" "powc:" "base:--tpke-pipeline 2" ...
set -o pipefail
TAG=${1:-ab}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
B="--steps 20 --warmup 5 --tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline"
shift
i=0
for spec in "$@"; do
  i=$((i+1))
  lib=${spec%%:*}; flags=${spec#*:}
  if [[ $lib == base ]]; then unset LCB_LIB_PATH; else export LCB_LIB_PATH=$R/lachain_amd/abv/$lib/liblachain_bls.so; fi
  out=gpurun_out/$TAG/run$i
  timeout -k 10 240 python -u bench.py $B $flags > $out.txt 2> $out.err || { echo "FAILED $spec"; tail -5 $out.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '|', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],2), 'ms/step, single', round(d['config'].get('single_batch_latency_ms') or 0, 2), 'ms, hwq', d['config'].get('hw_queues'))" $out.txt "$spec"
done
echo done
