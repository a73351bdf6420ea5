#!/bin/bash
# kernel stats, deterministic mode vs default (where the 4.6 % goes)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3x
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
for d in 1 0; do
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/p$d -o run -- python3 $R/bench.py --steps 3 --warmup 4 --deterministic $d > $O/p$d.txt 2>&1 || { tail -20 $O/p$d.txt; exit 1; }
done
cd $R
for d in 1 0; do
T=$(ls $O/p$d/*/run_kernel_trace.csv $O/p$d/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/kernel_stats.py $T --step-marker sgd --last 3 --top 40 > $O/stats_det$d.txt
rm -rf $O/p$d
head -25 $O/stats_det$d.txt | cut -c1-120
done
