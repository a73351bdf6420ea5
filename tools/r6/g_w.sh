#!/bin/bash
# saved-tensor hand-over warming: BERT-base A/B MIPIPE_PREFETCH=w (weights + hand-over) vs w (weights only)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=.
B="--model bert_base --seq 128 --steps 30 --warmup 5 --reference-config off --time-deterministic off"
for r in 1 2 3; do
  MIPIPE_PREFETCH=w timeout -k 10 300 python bench.py $B >> $O/g_w_w.jsonl 2>/dev/null || exit 1
  MIPIPE_PREFETCH=w0 timeout -k 10 300 python bench.py $B >> $O/g_w_w0.jsonl 2>/dev/null || exit 1
done
python -c "import json;[print(t, json.loads(l)['value']) for t in ('w','w0') for l in open('$O/g_w_%s.jsonl'%t) if l.startswith('{')]"
