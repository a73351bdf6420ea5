#!/bin/bash
# BERT-base A/B: GELU in the FFN-in GEMM epilogue (MIPIPE_GEMM_GELU=1) vs separate pass
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
B="--model bert_base --seq 128 --steps 30 --warmup 5 --reference-config off --time-deterministic off"
for r in 1 2 3; do
  for g in 1 0; do
    MIPIPE_GEMM_GELU=$g timeout -k 10 300 python bench.py $B > $O/g_gelu_$g.$r.json 2>/dev/null || exit 1
    python -c "import json;print('gemm_gelu=$g', json.loads(open('$O/g_gelu_$g.$r.json').read().strip().splitlines()[-1])['value'])"
  done
done
