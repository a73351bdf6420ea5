#!/bin/bash
# GEMM operand prefetch: tests, BERT-base A/B (MIPIPE_PREFETCH auto vs 0), BERT trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_prefetch_gpu.py tests/test_attention_gpu.py tests/test_kernels_gpu.py -k "prefetch or touch or bert or gemm" > $O/g_pf4_tests.txt 2>&1; rc=$?
tail -3 $O/g_pf4_tests.txt
[ $rc -eq 0 ] || exit 1
B="--model bert_base --seq 128 --steps 30 --warmup 5 --reference-config off --time-deterministic off"
for r in 1 2; do
  timeout -k 10 300 python bench.py $B >> $O/g_pf4_on.jsonl 2>/dev/null || exit 1
  MIPIPE_PREFETCH=0 timeout -k 10 300 python bench.py $B >> $O/g_pf4_off.jsonl 2>/dev/null || exit 1
done
python -c "import json;[print(t, json.loads(l)['value']) for t in ('on','off') for l in open('$O/g_pf4_%s.jsonl'%t) if l.startswith('{')]"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p_pf4_bert -o run -- python bench.py --model bert_base --seq 128 --steps 5 --warmup 3 --reference-config off --time-deterministic off > $O/p_pf4_bert.log 2>&1 || exit 1
echo done
