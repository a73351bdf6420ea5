#!/bin/bash
# GELU epilogue A/B (MIPIPE_GEMM_GELU=0: GEMM + gelu_fwd pass), BERT 32x128 interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3zf
mkdir -p $O
cd $R
for i in 1 2 3; do
timeout -k 10 300 python3 bench.py --model bert_base --steps 40 > $O/bert_on_$i.txt 2>&1 || { tail -20 $O/bert_on_$i.txt; exit 1; }
echo "on  $(tail -1 $O/bert_on_$i.txt | cut -c60-130)"
MIPIPE_GEMM_GELU=0 timeout -k 10 300 python3 bench.py --model bert_base --steps 40 > $O/bert_off_$i.txt 2>&1 || { tail -20 $O/bert_off_$i.txt; exit 1; }
echo "off $(tail -1 $O/bert_off_$i.txt | cut -c60-130)"
done
