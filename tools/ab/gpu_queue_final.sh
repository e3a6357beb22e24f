#!/bin/bash
# the aggregation queue on the final build: default workers (3), 1 ms deadline, 16 and 64 one-share callers, twice
set -o pipefail
TAG=${1:-qfinal}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd $R
for rep in 1 2; do
  timeout -k 10 200 python3 -u tools/queue_bench.py --seconds 3 --deadlines 1 > gpurun_out/$TAG/q_$rep.jsonl 2> gpurun_out/$TAG/q_$rep.err || { echo "rep $rep failed"; tail -5 gpurun_out/$TAG/q_$rep.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/$TAG/q_$rep.jsonl'):
    d=json.loads(l); print('rep$rep', d['callers'], '%.0f' % d['shares_per_s'], 'p50 %.2f p90 %.2f' % (d['latency_ms']['p50'], d['latency_ms']['p90']), 'batch %.1f' % d['mean_batch'], d['decision_mismatches'])"
done
echo done
