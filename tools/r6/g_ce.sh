#!/bin/bash
# Split cross-entropy + LayerNorm default mode 8: tests, BERT-base bench x3, BERT kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_attention_gpu.py tests/test_fp32_gpu.py tests/test_model_gpu.py -k "layernorm or cross_entropy or bert or resnet" > $O/g_ce_tests.txt 2>&1; rc=$?
tail -3 $O/g_ce_tests.txt
[ $rc -eq 0 ] || exit 1
B="--model bert_base --seq 128 --steps 30 --warmup 5 --reference-config off --time-deterministic off"
for r in 1 2 3; do
  timeout -k 10 300 python bench.py $B >> $O/g_ce_bert.jsonl 2>/dev/null || exit 1
done
python -c "import json;[print('bert', json.loads(l)['value']) for l in open('$O/g_ce_bert.jsonl') if l.startswith('{')]"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p_ce_bert -o run -- python bench.py --model bert_base --seq 128 --steps 5 --warmup 3 --reference-config off --time-deterministic off > $O/p_ce_bert.log 2>&1 || exit 1
echo done
