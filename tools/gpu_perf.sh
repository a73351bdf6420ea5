#!/bin/bash
# perf iteration: kernel tests, bench, per-layer conv microbench, kernel profile
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -x > gpurun_out/gpu_tests.txt 2>&1
rc=$?
tail -2 gpurun_out/gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.txt 2>&1 || exit $?
tail -1 gpurun_out/bench.txt
if [ "${MICRO:-1}" = "1" ]; then
  timeout -k 10 300 python tools/bench_kernels.py --iters 10 > gpurun_out/microbench.jsonl 2>&1 || exit $?
  tail -1 gpurun_out/microbench.jsonl
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --graph off > $R/gpurun_out/prof_bench.txt 2>&1 || exit $?
echo "prof ok"
