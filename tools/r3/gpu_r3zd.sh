#!/bin/bash
# one-level fixed-order column sums up to 1024 rows (BERT LayerNorm parameter grads): A/B vs the
# two-level threshold of 256 rows, BERT and deterministic ResNet-50
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3zd
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_determinism_gpu.py tests/test_attention_gpu.py tests/test_kernels_gpu.py -k "det or layernorm or attention or bert" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --model bert_base --steps 30 > $O/bert_new_$i.txt 2>&1 || { tail -20 $O/bert_new_$i.txt; exit 1; }
  echo "bert new $(tail -1 $O/bert_new_$i.txt | cut -c60-130)"
  MIPIPE_DET_TWO_LEVEL_ROWS=256 timeout -k 10 300 python3 bench.py --model bert_base --steps 30 > $O/bert_old_$i.txt 2>&1 || { tail -20 $O/bert_old_$i.txt; exit 1; }
  echo "bert old $(tail -1 $O/bert_old_$i.txt | cut -c60-130)"
done
timeout -k 10 300 python3 bench.py --steps 30 --deterministic 1 > $O/r50det_new.txt 2>&1 || { tail -20 $O/r50det_new.txt; exit 1; }
echo "r50 det new $(tail -1 $O/r50det_new.txt | cut -c60-130)"
MIPIPE_DET_TWO_LEVEL_ROWS=256 timeout -k 10 300 python3 bench.py --steps 30 --deterministic 1 > $O/r50det_old.txt 2>&1 || { tail -20 $O/r50det_old.txt; exit 1; }
echo "r50 det old $(tail -1 $O/r50det_old.txt | cut -c60-130)"
