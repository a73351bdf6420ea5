#!/bin/bash
# tiny-table embedding backward: tests, BERT-base bench x2, trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_attention_gpu.py -k "embedding or bert" > $O/g_emb3_tests.txt 2>&1; rc=$?
tail -3 $O/g_emb3_tests.txt
[ $rc -eq 0 ] || exit 1
B="--model bert_base --seq 128 --steps 30 --warmup 5 --reference-config off --time-deterministic off"
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > $O/g_emb3_bert.$r.json 2>/dev/null || exit 1
  python -c "import json;print('bert', json.loads(open('$O/g_emb3_bert.$r.json').read().strip().splitlines()[-1])['value'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p_emb3_bert -o run -- python bench.py --model bert_base --seq 128 --steps 5 --warmup 3 --reference-config off --time-deterministic off > $O/p_emb3_bert.log 2>&1 || exit 1
echo done
