#!/bin/bash
# PMC counters of the patch-resident 3x3 weight-grad at ResNet-50 layer1 / layer3 shapes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU"
G2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
for spec in "256 56 64 64 3 1 1 wgrad:l1" "256 14 256 256 3 1 1 wgrad:l3"; do
  args=${spec%:*}; tag=${spec##*:}
  gi=0
  for grp in "$G1" "$G2"; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/${tag}_$gi -o run -- python3 $R/tools/one_conv.py $args > $O/log_${tag}_$gi.txt 2>&1 || { echo "pmc $tag $gi failed"; tail -3 $O/log_${tag}_$gi.txt; exit 1; }
    gi=$((gi+1))
  done
  python3 $R/tools/r3/pmc_summary.py wgrad3x3 $O/${tag}_0 $O/${tag}_1 > $O/summary_$tag.txt
  echo "== $tag"; cat $O/summary_$tag.txt
  rm -rf $O/${tag}_0 $O/${tag}_1
done
