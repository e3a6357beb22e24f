#!/bin/bash
# Stall-breakdown PMC passes over the TPKE verify and TS verify kernels.  Usage: bash tools/pmc_stall.sh TAG
set -o pipefail
TAG=${1:-stall}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --shares 262144 --steps 1 --warmup 0 --no-cpu-baseline --ts-rounds 2621 --ts-steps 1 --msm-sizes "" --replay-n 0"
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_CYCLES"
G2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_WAVES"
i=0
for grp in "$G1" "$G2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${TAG}_$i -o run -- $CMD > $R/gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $R/gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
echo done
