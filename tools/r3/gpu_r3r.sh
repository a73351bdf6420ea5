#!/bin/bash
# which change moved BERT graphed-vs-eager: split-K plans, AdamW grid, or neither (run the test alone)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3r
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
T=tests/test_attention_gpu.py::test_bert_graphed_step_matches_eager
for cfg in "1 32768" "0 32768" "1 8192" "0 8192"; do
  set -- $cfg
  MIPIPE_GEMM_SPLITK=$1 MIPIPE_ADAMW_BLOCKS=$2 timeout -k 10 200 python3 -u -m pytest -q -x --timeout 150 --timeout-method thread $T > $O/t_$1_$2.txt 2>&1
  echo "splitk=$1 adamw_blocks=$2 rc=$? $(grep -E 'passed|failed' $O/t_$1_$2.txt | tail -1)"
  grep -E "^E .*\[\(" $O/t_$1_$2.txt | cut -c1-400 | head -3
done
timeout -k 10 300 python3 -u -m pytest -q -x --timeout 150 --timeout-method thread tests/test_attention_gpu.py > $O/attn_file.txt 2>&1
echo "whole file rc=$? $(tail -1 $O/attn_file.txt)"
grep -E "^E .*\[\(" $O/attn_file.txt | cut -c1-600 | head -3
exit 0
