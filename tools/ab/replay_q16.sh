#!/bin/bash
# The round-5 abort configuration on this build: 8 hardware queues per priority (Q = 16), the TPKE pipeline followed by
# the concurrent epoch replay, under rocprofv3 (kernel trace).  Usage: bash tools/ab/replay_q16.sh TAG
set -o pipefail
TAG=${1:-q16}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/rocprof -o run -- python3 $R/bench.py --hw-queues 8 --no-cpu-baseline --pattern-steps 1 --mcl-reps 10 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --msm-sizes= > $R/gpurun_out/$TAG/bench_under_rocprof.txt 2>&1 || { echo "ROCPROF FAILED rc=$?"; tail -8 $R/gpurun_out/$TAG/bench_under_rocprof.txt; exit 1; }
grep -h "epoch replay\|threshold" $R/gpurun_out/$TAG/bench_under_rocprof.txt | head -3
python3 -c "
import json,sys
l=[x for x in open('$R/gpurun_out/$TAG/bench_under_rocprof.txt') if x.startswith('{')][-1]
d=json.loads(l); print('headline', d['value'], 'hwq', d['config'].get('hw_queues'), 'replay', d['summary'].get('epoch_replay'))
"
rm -f $R/gpurun_out/$TAG/rocprof/run_kernel_trace.csv
echo done
