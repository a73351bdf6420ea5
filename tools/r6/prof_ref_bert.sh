#!/bin/bash
# kernel stats of the reference config (ResNet-18 32^2 fp32 deterministic, 1000 classes, b1024)
# and of BERT-base 32x128 on the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_ref -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet18 --res 32 --classes 1000 --dtype fp32 --deterministic 1 --batch 1024 --steps 5 --warmup 5 --reference-config off --time-deterministic off > $O/p_ref.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_bert -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model bert_base --seq 128 --steps 5 --warmup 5 --reference-config off --time-deterministic off > $O/p_bert.log 2>&1 || exit 1
echo done
