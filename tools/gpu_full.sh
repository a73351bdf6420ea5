#!/bin/bash
# One GPU call: full GPU test suite, ResNet-50 + BERT benches, ResNet-50 kernel profile,
# then the 3-step pipeline rehearsal.  Every GPU step has its own time limit; stop on faults.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 600 python -m pytest tests/ -q -m gpu > gpurun_out/gpu_tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_tests.txt
tail -4 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.txt 2>&1 || exit $?
tail -1 gpurun_out/bench.txt
timeout -k 10 300 python bench.py --model bert_base --steps 10 --warmup 3 > gpurun_out/bench_bert.txt 2>&1 || exit $?
tail -1 gpurun_out/bench_bert.txt
if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --graph off > $R/gpurun_out/prof_bench.txt 2>&1 || exit $?
  echo "prof ok"
  cd $R
fi
if [ "${SKIP_PIPE:-0}" != "1" ]; then
  bash tools/gpu_pipeline.sh || exit $?
fi
