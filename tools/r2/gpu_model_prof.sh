#!/bin/bash
# Eager kernel trace of one zoo model's training step -> per-kernel-family stats.
# usage: bash tools/r2/gpu_model_prof.sh <model> [bench.py args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2
M=$1; shift
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$M -o run -- python3 $R/bench.py --model $M --steps 3 --warmup 3 --graph off "$@" > $O/prof_$M.txt 2>&1 || { tail -20 $O/prof_$M.txt; exit 1; }
cd $R
T=$(ls $O/prof_$M/*/run_kernel_trace.csv $O/prof_$M/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/kernel_stats.py $T --step-marker sgd --last 3 --top 30 > $O/stats_$M.txt
cat $O/stats_$M.txt
