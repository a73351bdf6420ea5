#!/bin/bash
# PMC counters for the short-K streaming conv (ResNet-50 layer1 1x1 64->256 forward) per tile.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r2/pmc_sk
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU"
G2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
for cfg in 1 9 0; do
  gi=0
  for grp in "$G1" "$G2"; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/c${cfg}_$gi -o run -- python3 $R/tools/one_conv.py 256 56 64 256 1 1 0 fwd $cfg > $O/log_${cfg}_$gi.txt 2>&1 || { echo "pmc $cfg $gi failed"; tail -3 $O/log_${cfg}_$gi.txt; exit 1; }
    gi=$((gi+1))
  done
  echo "done $cfg"
done
