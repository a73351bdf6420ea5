#!/bin/bash
# saved-tensor hand-over warming: BERT-base A/B MIPIPE_PREFETCH=1 (weights + hand-over) vs w (weights only)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=.
B="--model bert_base --seq 128 --steps 30 --warmup 5 --reference-config off --time-deterministic off"
for r in 1 2 3; do
  MIPIPE_PREFETCH=1 timeout -k 10 300 python bench.py $B >> $O/g_ho_full.jsonl 2>/dev/null || exit 1
  MIPIPE_PREFETCH=w timeout -k 10 300 python bench.py $B >> $O/g_ho_w.jsonl 2>/dev/null || exit 1
done
python -c "import json;[print(t, json.loads(l)['value']) for t in ('full','w') for l in open('$O/g_ho_%s.jsonl'%t) if l.startswith('{')]"
