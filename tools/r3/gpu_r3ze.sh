#!/bin/bash
# GELU epilogue (FFN up-projection stores h and gelu(h)): numerics, BERT throughput
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3ze
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python3 -u -m pytest -q -x --timeout 240 --timeout-method thread tests/test_attention_gpu.py tests/test_model_gpu.py -k "bert or attention or gelu or linear" > $O/tests_attn.txt 2>&1 || { tail -30 $O/tests_attn.txt; exit 1; }
tail -1 $O/tests_attn.txt
for i in 1 2; do
timeout -k 10 300 python3 bench.py --model bert_base --steps 30 > $O/bert_$i.txt 2>&1 || { tail -20 $O/bert_$i.txt; exit 1; }
echo "bert $(tail -1 $O/bert_$i.txt | cut -c60-130)"
done
timeout -k 10 300 python3 bench.py --model bert_base --batch 8 --seq 512 --steps 20 > $O/bert512.txt 2>&1 || { tail -20 $O/bert512.txt; exit 1; }
echo "bert512 $(tail -1 $O/bert512.txt | cut -c60-130)"
