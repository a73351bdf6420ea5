#!/bin/bash
# native C++ DDP reducer + bf16 wire kernels on RCCL (world 1, force_reduce), eager and graphed
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3l
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 600 python3 -u -m pytest -v -x --timeout 200 --timeout-method thread tests/test_ddp_gpu.py tests/test_task_gpu.py > $O/ddp_tests.txt 2>&1 || { tail -60 $O/ddp_tests.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/ddp_tests.txt | tail -20
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0
for r in 1 0; do
  MIPIPE_NATIVE_REDUCER=$r timeout -k 10 240 python3 bench.py --force-reduce --graph off --steps 20 --warmup 5 > $O/bench_fr_eager_native$r.txt 2>&1 || { tail -20 $O/bench_fr_eager_native$r.txt; exit 1; }
  tail -1 $O/bench_fr_eager_native$r.txt | cut -c1-200
done
timeout -k 10 240 python3 bench.py --force-reduce --graph on --steps 20 --warmup 5 > $O/bench_fr_graph.txt 2>&1 || { tail -20 $O/bench_fr_graph.txt; exit 1; }
tail -1 $O/bench_fr_graph.txt | cut -c1-200
