#!/bin/bash
# Comm/compute overlap: eager vs hipGraph replay, default vs high-priority side stream, and the
# HIP graph-queue count (DEBUG_HIP_FORCE_GRAPH_QUEUES) — wall-clock method, no tracer.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
for c in conv matmul; do
  for p in 0 -1; do
    timeout -k 10 120 python3 tools/r3/overlap_probe.py --compute $c --prio $p --gemms 40 --mb 256 > $O/ovl_${c}_p$p.txt 2>&1 || { tail -20 $O/ovl_${c}_p$p.txt; exit 1; }
    tail -1 $O/ovl_${c}_p$p.txt
  done
done
for q in 1 2 4 8; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 120 python3 tools/r3/overlap_probe.py --compute conv --gemms 40 --mb 256 > $O/ovl_q$q.txt 2>&1 || { tail -20 $O/ovl_q$q.txt; exit 1; }
  tail -1 $O/ovl_q$q.txt
done
TORCH_NCCL_HIGH_PRIORITY=1 timeout -k 10 120 python3 tools/r3/overlap_probe.py --compute conv --gemms 40 --mb 256 > $O/ovl_hp.txt 2>&1 || { tail -20 $O/ovl_hp.txt; exit 1; }
tail -1 $O/ovl_hp.txt
