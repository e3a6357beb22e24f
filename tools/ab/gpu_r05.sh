#!/bin/bash
# Round 5 GPU step: environment facts, the full GPU suite, then the default bench run (every exit status checked; a
# failed step ends the call).  Usage: bash tools/gpu_r05.sh TAG [bench args]
set -o pipefail
TAG=${1:-r05}; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
{ echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset}"; grep -h -E "max_slots_scratch_cu|max_waves_per_simd|simd_count|array_count|cu_per_simd_array" /sys/class/kfd/kfd/topology/nodes/*/properties 2>/dev/null | sort | uniq -c; } > gpurun_out/$TAG/env.txt
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.txt 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/$TAG/tests.txt; exit 1; }
  tail -3 gpurun_out/$TAG/tests.txt
fi
timeout -k 10 900 python -u bench.py "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "BENCH FAILED"; tail -30 gpurun_out/$TAG/bench.err; exit 1; }
tail -c 6000 gpurun_out/$TAG/bench.json
