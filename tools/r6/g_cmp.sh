#!/bin/bash
# same-box comparators: mipipe vs stock PyTorch-ROCm (ResNet-50, BERT-base 32x128, BERT-base 8x512,
# the reference config fp32 deterministic)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
R="--reference-config off --time-deterministic off"
REF="--model resnet18 --res 32 --classes 1000 --dtype fp32 --deterministic 1 --batch 1024"
n=0
run() { n=$((n+1)); timeout -k 10 400 python -u bench.py "$@" > $O/f_cmp_$n.json 2> $O/f_cmp_$n.err || return 1; tail -1 $O/f_cmp_$n.json | cut -c1-120; }
run $R || exit 1
run $R --impl stock || exit 1
run $R --model bert_base --seq 128 || exit 1
run $R --model bert_base --seq 128 --impl stock || exit 1
run $R --model bert_base --seq 512 --batch 8 || exit 1
run $R --model bert_base --seq 512 --batch 8 --impl stock || exit 1
run $R $REF || exit 1
run $R $REF --impl stock || exit 1
echo done
