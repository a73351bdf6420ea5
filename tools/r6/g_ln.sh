#!/bin/bash
# LayerNorm exact-width kernels: tests, per-kernel timings, BERT-base A/B (generic vs exact)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_attention_gpu.py -k "layernorm or bert" > $O/g_ln_tests.txt 2>&1; rc=$?
tail -3 $O/g_ln_tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/r6/ln_bench.py > $O/g_ln_bench.jsonl 2>&1 || exit 1
cat $O/g_ln_bench.jsonl
for r in 1 2; do
  MIPIPE_LN_MODE=16 timeout -k 10 300 python bench.py --model bert_base --seq 128 --steps 30 --warmup 5 --reference-config off --time-deterministic off >> $O/g_ln_bert16.jsonl 2>/dev/null || exit 1
  MIPIPE_LN_MODE=0 timeout -k 10 300 python bench.py --model bert_base --seq 128 --steps 30 --warmup 5 --reference-config off --time-deterministic off >> $O/g_ln_bert0.jsonl 2>/dev/null || exit 1
done
python -c "import json;[print(t, json.loads(l)['value']) for t in ('16','0') for l in open('$O/g_ln_bert%s.jsonl'%t) if l.startswith('{')]"
echo done
