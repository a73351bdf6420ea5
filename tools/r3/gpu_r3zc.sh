#!/bin/bash
# BERT-base 32x128 kernel profile (graph replay) after the library GEMM plans
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3zc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pr -o run -- python3 $R/bench.py --model bert_base --steps 3 --warmup 4 > $O/pr.txt 2>&1 || { tail -20 $O/pr.txt; exit 1; }
cd $R
T=$(ls $O/pr/*/run_kernel_trace.csv $O/pr/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/r2/per_call.py $T --marker adamw > $O/bert_calls.txt
python3 tools/kernel_stats.py $T --step-marker adamw --last 3 --top 30 > $O/bert_stats.txt
rm -rf $O/pr
cat $O/bert_stats.txt
