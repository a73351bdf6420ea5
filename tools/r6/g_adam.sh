#!/bin/bash
# AdamW items in flight per thread: tests, BERT-base A/B MIPIPE_ADAMW_UNROLL 2 vs 1
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
MIPIPE_ADAMW_UNROLL=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_optim_ddp.py tests/test_attention_gpu.py -k "adamw or sgd or bert" -m gpu > $O/g_adam_tests.txt 2>&1; rc=$?
tail -2 $O/g_adam_tests.txt
[ $rc -eq 0 ] || exit 1
B="--model bert_base --seq 128 --steps 30 --warmup 5 --reference-config off --time-deterministic off"
for r in 1 2 3; do
  for u in 4 2; do
    MIPIPE_ADAMW_UNROLL=$u timeout -k 10 300 python bench.py $B > $O/g_adam4_$u.$r.json 2>/dev/null || exit 1
    python -c "import json;print('unroll=$u', json.loads(open('$O/g_adam4_$u.$r.json').read().strip().splitlines()[-1])['value'])"
  done
done
