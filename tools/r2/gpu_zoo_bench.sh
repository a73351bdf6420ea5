#!/bin/bash
# Zoo throughput on one MI355X (bf16, synthetic, 224² / 299² Inception), mipipe kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
: > $O/zoo_bench.jsonl
for m in mobilenet_v2 resnext50_32x4d densenet121 shufflenet_v2_x1_0 vgg16 resnet101 wide_resnet50_2; do
  timeout -k 10 300 python3 $R/bench.py --model $m --steps 10 --warmup 4 > $O/zb_$m.txt 2>&1 || { tail -20 $O/zb_$m.txt; exit 1; }
  tail -1 $O/zb_$m.txt >> $O/zoo_bench.jsonl; echo "$m $(tail -1 $O/zb_$m.txt | cut -c95-150)"
done
timeout -k 10 300 python3 $R/bench.py --model inception_v3 --res 299 --batch 128 --steps 10 --warmup 4 > $O/zb_inception.txt 2>&1 || { tail -20 $O/zb_inception.txt; exit 1; }
tail -1 $O/zb_inception.txt >> $O/zoo_bench.jsonl; echo "inception $(tail -1 $O/zb_inception.txt | cut -c95-150)"
