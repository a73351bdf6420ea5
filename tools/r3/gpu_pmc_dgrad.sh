#!/bin/bash
# per-dispatch PMC of the ResNet-50 step's longest data-grads (fused BN-backward epilogues)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY"
gi=0
for grp in "$G1" "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/dg_$gi -o run -- python3 $R/bench.py --steps 1 --warmup 4 --graph off > $O/log_dg_$gi.txt 2>&1 || { echo "pmc $gi failed"; tail -5 $O/log_dg_$gi.txt; exit 1; }
  gi=$((gi+1))
done
python3 $R/tools/r3/pmc_dispatch.py conv_dgrad 8 $O/dg_0 $O/dg_1 $O/dg_2 | tee $O/dgrad_dispatch.txt
python3 $R/tools/r3/pmc_dispatch.py bn_bwd_apply 3 $O/dg_0 $O/dg_1 $O/dg_2 | tee -a $O/dgrad_dispatch.txt
python3 $R/tools/r3/pmc_dispatch.py bn_act_fwd 2 $O/dg_0 $O/dg_1 $O/dg_2 | tee -a $O/dgrad_dispatch.txt
rm -rf $O/dg_0 $O/dg_1 $O/dg_2
