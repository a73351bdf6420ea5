#!/bin/bash
# Conv kernel tests, then the headline + secondary benches (ResNet-50 b256 bf16, BERT-base MLM
# 32x128 / 8x512, ResNet-18 CIFAR-shape fp32 b1024) and the ResNet-50 per-call profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or production" > $O/bench_tests.txt 2>&1 || { tail -30 $O/bench_tests.txt; exit 1; }
tail -1 $O/bench_tests.txt
run() { local name=$1; shift; timeout -k 10 300 python3 $R/bench.py "$@" > $O/b_$name.txt 2>&1 || { tail -20 $O/b_$name.txt; exit 1; }; echo "$name $(tail -1 $O/b_$name.txt)"; }
run r50 --steps 20 --warmup 5
run bert128 --model bert_base --steps 10 --warmup 3
run bert512 --model bert_base --seq 512 --batch 8 --steps 10 --warmup 3
run r18fp32 --model resnet18 --res 32 --batch 1024 --classes 10 --dtype fp32 --steps 30 --warmup 5
bash $R/tools/r2/gpu_percall.sh
