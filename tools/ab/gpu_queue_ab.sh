#!/bin/bash
# queue bench at 2 / 3 / 4 workers (LCB_QUEUE_WORKERS), 1 ms deadline, 16 and 64 one-share callers, twice each
set -o pipefail
TAG=${1:-qab}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd $R
for rep in 1 2; do
  for w in 2 3 4; do
    LCB_QUEUE_WORKERS=$w timeout -k 10 200 python3 -u tools/queue_bench.py --seconds 3 --deadlines 1 > gpurun_out/$TAG/w${w}_$rep.jsonl 2> gpurun_out/$TAG/w${w}_$rep.err || { echo "w$w failed"; tail -5 gpurun_out/$TAG/w${w}_$rep.err; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/$TAG/w${w}_$rep.jsonl'):
    d=json.loads(l); print('w$w', d['callers'], '%.0f' % d['shares_per_s'], 'p50 %.2f p90 %.2f' % (d['latency_ms']['p50'], d['latency_ms']['p90']), 'batch %.1f' % d['mean_batch'], d['decision_mismatches'])"
  done
done
