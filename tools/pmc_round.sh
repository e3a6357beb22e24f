#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over a 262,144-share bench launch.  Usage: bash tools/pmc_round.sh TAG
set -o pipefail
TAG=${1:-pmc}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
CMD=${PMC_CMD:-"python3 $R/bench.py --shares 262144 --steps 1 --warmup 0 --no-cpu-baseline --ts-rounds 4096 --msm-steps 1 --msm-sizes 1048576 --replay-n 0 --ecdsa-sigs 262144 --ecdsa-steps 1 --dkg-n 0 --rs-n 0"}
i=0
PMC_GROUPS=${PMC_GROUPS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU;FETCH_SIZE;WRITE_SIZE"}
IFS=';' read -ra GRPS <<< "$PMC_GROUPS"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${TAG}_$i -o run -- $CMD > $R/gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $R/gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
echo done
