#!/bin/bash
# PMC counters for one conv shape (counters only with kernel-trace; no sys/runtime traces)
set -o pipefail
OUT=${OUT:-pmc}
mkdir -p gpurun_out/$OUT
R=$PWD
SHAPE="${SHAPE:-256 14 256 256 3 1 1 fwd}"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $R/gpurun_out/$OUT/g$i -o run -- python3 $R/tools/one_conv.py $SHAPE > $R/gpurun_out/$OUT/log$i.txt 2>&1 || { echo "pmc group $i failed"; tail -5 $R/gpurun_out/$OUT/log$i.txt; }
  i=$((i+1))
done
ls -R $R/gpurun_out/$OUT | head -30
