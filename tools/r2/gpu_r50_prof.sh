#!/bin/bash
# ResNet-50 b256 kernel trace (eager, tuned tiles) -> per-kernel-family time per step.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/prof_r50 -o run -- python3 $R/bench.py --steps 4 --warmup 4 --graph off > $O/prof_r50.txt 2>&1 || { tail -20 $O/prof_r50.txt; exit 1; }
cd $R
python3 tools/kernel_stats.py $O/prof_r50/run_kernel_trace.csv --step-marker sgd --last 3 --top 45 > $O/r50_kernel_stats.txt
cat $O/r50_kernel_stats.txt
