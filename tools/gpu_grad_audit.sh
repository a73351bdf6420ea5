#!/bin/bash
# gradient audit of the zoo on one GPU (see tools/grad_audit.py)
set -o pipefail
mkdir -p gpurun_out
CFGS="${AUDIT:-resnet18 32;mobilenet_v2 64;mnasnet0_5 64;shufflenet_v2_x1_0 64;resnext50_32x4d 64;googlenet 64;densenet121 64;squeezenet1_1 64;inception_v3 299}"
IFS=';' read -ra LIST <<< "$CFGS"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  echo "== $1 $2" >> gpurun_out/grad_audit.txt
  timeout -k 10 200 python -u tools/grad_audit.py --arch $1 --res $2 $AUDIT_FLAGS >> gpurun_out/grad_audit.txt 2>&1 \
    || { echo "FAILED $1"; tail -5 gpurun_out/grad_audit.txt; exit 1; }
  grep -E "^AUDIT|^STOCK|^train-mode" gpurun_out/grad_audit.txt | tail -3
done
