#!/bin/bash
# profiles: BERT-base 32x128 (graph replay) kernel stats; ResNet-50 b256 per-call trace (current code)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3o
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 300 python3 bench.py --model bert_base --steps 30 > $O/bert128.txt 2>&1 || { tail -20 $O/bert128.txt; exit 1; }
tail -1 $O/bert128.txt | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pb -o run -- python3 $R/bench.py --model bert_base --steps 5 --warmup 3 > $O/pb.txt 2>&1 || { tail -20 $O/pb.txt; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pr -o run -- python3 $R/bench.py --steps 3 --warmup 4 > $O/pr.txt 2>&1 || { tail -20 $O/pr.txt; exit 1; }
cd $R
T=$(ls $O/pb/*/run_kernel_trace.csv $O/pb/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/kernel_stats.py $T --step-marker adamw --last 5 --top 40 > $O/bert128_stats.txt
python3 tools/r2/per_call.py $T > $O/bert128_calls.txt
T=$(ls $O/pr/*/run_kernel_trace.csv $O/pr/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/kernel_stats.py $T --step-marker sgd --last 3 --top 45 > $O/r50_stats.txt
python3 tools/r2/per_call.py $T > $O/r50_calls.txt
rm -rf $O/pb $O/pr
head -30 $O/bert128_stats.txt
head -8 $O/r50_stats.txt
