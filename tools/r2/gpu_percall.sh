#!/bin/bash
# ResNet-50 b256 bf16: 1-GPU bench (graph replay) + eager kernel trace -> per-call listing of one step.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 > $O/pc_bench.txt 2>&1 || { tail -20 $O/pc_bench.txt; exit 1; }
tail -1 $O/pc_bench.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_pc -o run -- python3 $R/bench.py --steps 3 --warmup 4 --graph off > $O/pc_prof.txt 2>&1 || { tail -20 $O/pc_prof.txt; exit 1; }
cd $R
T=$(ls $O/prof_pc/*/run_kernel_trace.csv $O/prof_pc/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/r2/per_call.py $T > $O/pc_calls.txt
python3 tools/kernel_stats.py $T --step-marker sgd --last 3 --top 30 > $O/pc_stats.txt
head -3 $O/pc_stats.txt
