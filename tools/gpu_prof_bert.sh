#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bert -o run -- python3 $R/bench.py --model bert_base --steps 5 --warmup 2 > $R/gpurun_out/prof_bert.txt 2>&1 || exit $?
tail -1 $R/gpurun_out/prof_bert.txt
timeout -k 10 300 python3 $R/bench.py --model bert_base --seq 512 --batch 8 --steps 10 --warmup 3 > $R/gpurun_out/bench_bert512.txt 2>&1 || exit $?
tail -1 $R/gpurun_out/bench_bert512.txt
timeout -k 10 300 python3 $R/bench.py --model bert_base --seq 512 --batch 8 --impl stock --steps 10 --warmup 3 > $R/gpurun_out/bench_bert512_stock.txt 2>&1 || exit $?
tail -1 $R/gpurun_out/bench_bert512_stock.txt
