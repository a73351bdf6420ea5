#!/bin/bash
# library (hipBLASLt) GEMM plan: numerics, per-shape timing, BERT / ResNet-50 throughput
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3zb
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k gemm > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python3 -u -m pytest -q -x --timeout 240 --timeout-method thread tests/test_attention_gpu.py > $O/tests_attn.txt 2>&1 || { tail -30 $O/tests_attn.txt; exit 1; }
tail -1 $O/tests_attn.txt
timeout -k 10 400 python3 -u tools/r3/gemm_vs_blaslt.py > $O/gemm.txt 2>&1 || { tail -30 $O/gemm.txt; exit 1; }
tail -3 $O/gemm.txt
for i in 1 2; do
timeout -k 10 300 python3 bench.py --model bert_base --steps 30 > $O/bert_$i.txt 2>&1 || { tail -20 $O/bert_$i.txt; exit 1; }
echo "bert $(tail -1 $O/bert_$i.txt | cut -c60-130)"
MIPIPE_GEMM_LIB=0 timeout -k 10 300 python3 bench.py --model bert_base --steps 30 > $O/bert_nolib_$i.txt 2>&1 || { tail -20 $O/bert_nolib_$i.txt; exit 1; }
echo "bert nolib $(tail -1 $O/bert_nolib_$i.txt | cut -c60-130)"
done
timeout -k 10 300 python3 bench.py --model bert_base --batch 8 --seq 512 --steps 20 > $O/bert512.txt 2>&1 || { tail -20 $O/bert512.txt; exit 1; }
echo "bert512 $(tail -1 $O/bert512.txt | cut -c60-130)"
timeout -k 10 300 python3 bench.py --steps 30 > $O/r50.txt 2>&1 || { tail -20 $O/r50.txt; exit 1; }
echo "r50 $(tail -1 $O/r50.txt | cut -c60-130)"
