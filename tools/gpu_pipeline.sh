#!/bin/bash
# BASELINE config 5 rehearsal on the 1-GPU box: preprocess -> train (launcher, 1 rank) -> eval
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export MIPIPE_GCS_ROOT=/tmp/mipipe_gcs
export MIPIPE_CACHE_DIR=/tmp/mipipe_cache
timeout -k 10 900 python examples/three_step_pipeline.py --gpus 1 --arch ${ARCH:-resnet18} --dataset cifar10 \
  --epochs 3 --n-train 20000 --n-test 2000 --batch-size 256 --lr 0.05 --baseline-accuracy 50 \
  --serving-dir /tmp/mipipe_serving --spec gpurun_out/three_step.json > gpurun_out/pipeline.txt 2>&1
rc=$?
tail -30 gpurun_out/pipeline.txt
find /tmp/mipipe_gcs -name "run.json" -exec cp {} gpurun_out/pipeline_run.json \;
find /tmp/mipipe_gcs -name "rank0.log" -exec cp {} gpurun_out/pipeline_rank0.log \;
ls -R /tmp/mipipe_serving | head -20
exit $rc
