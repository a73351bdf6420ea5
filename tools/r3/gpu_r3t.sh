#!/bin/bash
# fused dropout + residual LayerNorm: numerics tests, BERT graph test, BERT benches
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3t
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 400 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_attention_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
timeout -k 10 300 python3 bench.py --model bert_base --steps 30 > $O/bert128_$i.txt 2>&1 || { tail -20 $O/bert128_$i.txt; exit 1; }
tail -1 $O/bert128_$i.txt | cut -c1-160
done
timeout -k 10 300 python3 bench.py --model bert_base --seq 512 --batch 8 --steps 20 > $O/bert512.txt 2>&1 || { tail -20 $O/bert512.txt; exit 1; }
tail -1 $O/bert512.txt | cut -c1-160
