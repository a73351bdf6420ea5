#!/bin/bash
# PMC counters (own runs, kernel-trace only) for representative conv shapes / tile configs.
set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out/r2/pmc
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU"
G2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
G3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
for spec in "256 14 256 256 3 1 1 fwd 0:a" "256 14 256 256 3 1 1 fwd 6:b" "256 56 64 64 3 1 1 fwd 2:c" "256 56 64 64 3 1 1 dgrad 2:d" "256 14 1024 256 1 1 0 dgrad 1:e"; do
  args=${spec%:*}; tag=${spec##*:}
  gi=0
  for grp in "$G1" "$G2" "$G3"; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $R/gpurun_out/r2/pmc/$tag$gi -o run -- python3 $R/tools/one_conv.py $args > $R/gpurun_out/r2/pmc/log_$tag$gi.txt 2>&1 || { echo "pmc $tag $gi failed"; tail -3 $R/gpurun_out/r2/pmc/log_$tag$gi.txt; exit 1; }
    gi=$((gi+1))
  done
  echo "done $tag"
done
