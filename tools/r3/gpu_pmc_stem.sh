#!/bin/bash
# PMC counters of the recompute-fused stem kernels (stem.hip) at b256
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU"
G2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
gi=0
for grp in "$G1" "$G2"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/stem_$gi -o run -- python3 $R/tools/r3/stem_ab.py --iters 2 --modes 1 > $O/log_stem_$gi.txt 2>&1 || { echo "pmc $gi failed"; tail -5 $O/log_stem_$gi.txt; exit 1; }
  gi=$((gi+1))
done
for k in stem_stats stem_pool pool_bn_bwd_reduce stem_bwd_wgrad; do
  echo "== $k"
  python3 $R/tools/r3/pmc_summary.py $k $O/stem_0 $O/stem_1 | tee $O/summary_$k.txt
done
rm -rf $O/stem_0 $O/stem_1
