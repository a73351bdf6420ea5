#!/bin/bash
# tuner timing with cold caches (MIPIPE_TUNE_REPS=1) vs back-to-back: ResNet-50 and BERT-base A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
R="--reference-config off --time-deterministic off --steps 30 --warmup 5"
for r in 1 2; do
  for c in 10 3; do
    MIPIPE_TUNE_REPS=$c timeout -k 10 300 python bench.py $R > $O/g_reps_r50_$c.$r.json 2>/dev/null || exit 1
    python -c "import json;print('r50 reps=$c', json.loads(open('$O/g_reps_r50_$c.$r.json').read().strip().splitlines()[-1])['value'])"
    MIPIPE_TUNE_REPS=$c timeout -k 10 300 python bench.py $R --model bert_base --seq 128 > $O/g_reps_bert_$c.$r.json 2>/dev/null || exit 1
    python -c "import json;print('bert reps=$c', json.loads(open('$O/g_reps_bert_$c.$r.json').read().strip().splitlines()[-1])['value'])"
  done
done
