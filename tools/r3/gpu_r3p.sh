#!/bin/bash
# BERT GEMM split-K plans vs hipBLASLt, AdamW variant lab, BERT bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3p
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 120 ./tools/r3/adamw_lab > $O/adamw_lab.txt 2>&1 || { tail -20 $O/adamw_lab.txt; exit 1; }
cat $O/adamw_lab.txt
timeout -k 10 300 python3 tools/r3/gemm_vs_blaslt.py > $O/gemm.txt 2>&1 || { tail -20 $O/gemm.txt; exit 1; }
cat $O/gemm.txt
timeout -k 10 300 python3 bench.py --model bert_base --steps 30 > $O/bert128.txt 2>&1 || { tail -20 $O/bert128.txt; exit 1; }
tail -1 $O/bert128.txt | cut -c1-200
