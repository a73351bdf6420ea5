#!/bin/bash
# GPU check of the attention/BERT path + BERT bench (mipipe and stock comparator).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_attention_gpu.py -q -x > gpurun_out/attn_tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/attn_tests.txt
tail -15 gpurun_out/attn_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --model bert_base --steps 10 --warmup 3 > gpurun_out/bench_bert.txt 2>&1 || exit $?
tail -1 gpurun_out/bench_bert.txt
timeout -k 10 300 python bench.py --model bert_base --impl stock --steps 10 --warmup 3 > gpurun_out/bench_bert_stock.txt 2>&1 || exit $?
tail -1 gpurun_out/bench_bert_stock.txt
