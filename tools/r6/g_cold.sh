#!/bin/bash
# tuner timing with cold caches (MIPIPE_TUNE_COLD=1) vs back-to-back: ResNet-50 and BERT-base A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
R="--reference-config off --time-deterministic off --steps 30 --warmup 5"
for r in 1 2; do
  for c in 1 0; do
    MIPIPE_TUNE_COLD=$c timeout -k 10 300 python bench.py $R > $O/g_cold_r50_$c.$r.json 2>/dev/null || exit 1
    python -c "import json;print('r50 cold=$c', json.loads(open('$O/g_cold_r50_$c.$r.json').read().strip().splitlines()[-1])['value'])"
    MIPIPE_TUNE_COLD=$c timeout -k 10 300 python bench.py $R --model bert_base --seq 128 > $O/g_cold_bert_$c.$r.json 2>/dev/null || exit 1
    python -c "import json;print('bert cold=$c', json.loads(open('$O/g_cold_bert_$c.$r.json').read().strip().splitlines()[-1])['value'])"
  done
done
