#!/bin/bash
# First GPU call of round 2: GPU tests + smoke + 1-GPU bench, then RCCL/DDP path checks.
set -o pipefail
bash tools/r2/gpu_baseline.sh || exit $?
bash tools/r2/gpu_ddp.sh || exit $?
