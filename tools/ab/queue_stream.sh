#!/bin/bash
# Queue latency with ciphertext preparations arriving continuously, beside the prepare-ahead baseline.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/qs
for ps in 0 100 400; do
  timeout -k 10 200 python -u tools/queue_bench.py --deadlines 1 --threads 64 --seconds 4 --prepare-stream $ps > gpurun_out/qs/ps_$ps.jsonl 2> gpurun_out/qs/ps_$ps.err || { echo "FAILED $ps"; tail -5 gpurun_out/qs/ps_$ps.err; exit 1; }
  cat gpurun_out/qs/ps_$ps.jsonl
done
