#!/bin/bash
# GEMM vs hipBLASLt on the BERT shapes, graph-replay timing, incl. fp32-accumulate weight-grads
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3za
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u tools/r3/gemm_vs_blaslt.py > $O/gemm.txt 2>&1 || { tail -30 $O/gemm.txt; exit 1; }
cat $O/gemm.txt
