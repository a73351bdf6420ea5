#!/bin/bash
# BERT-base MLM 8x512: mipipe vs stock throughput, rocprofv3 kernel trace of the mipipe step,
# and the torch-profiler attribution of any remaining ATen kernels to their call sites.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r2
timeout -k 10 300 python3 $R/bench.py --model bert_base --seq 512 --batch 8 --steps 20 --warmup 5 > $O/bert512.txt 2>&1 || { tail -20 $O/bert512.txt; exit 1; }
tail -1 $O/bert512.txt
timeout -k 10 300 python3 $R/tools/prof_bert_aten.py 8 512 > $O/bert512_aten.txt 2>&1 || { tail -20 $O/bert512_aten.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_bert512 -o run -- python3 $R/bench.py --model bert_base --seq 512 --batch 8 --steps 5 --warmup 3 > $O/prof_bert512.txt 2>&1 || { tail -20 $O/prof_bert512.txt; exit 1; }
cd $R
python3 tools/kernel_stats.py $(ls $O/prof_bert512/*kernel_trace.csv | head -1) --step-marker adamw --last 5 --top 40 > $O/bert512_kernel_stats.txt
head -50 $O/bert512_kernel_stats.txt
if [ "${STOCK:-1}" = 1 ]; then
timeout -k 10 300 python3 $R/bench.py --model bert_base --seq 512 --batch 8 --impl stock --steps 20 --warmup 5 > $O/bert512_stock.txt 2>&1 || { tail -20 $O/bert512_stock.txt; exit 1; }
tail -1 $O/bert512_stock.txt
fi
