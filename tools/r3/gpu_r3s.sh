#!/bin/bash
# workspace split-K plans: GEMM plan tests, BERT wgrad probe, BERT benches
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3s
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 400 python3 -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > $O/gemm_tests.txt 2>&1 || { tail -30 $O/gemm_tests.txt; exit 1; }
tail -1 $O/gemm_tests.txt
timeout -k 10 300 python3 tools/r3/gemm_vs_blaslt.py > $O/gemm.txt 2>&1 || { tail -20 $O/gemm.txt; exit 1; }
grep wgrad $O/gemm.txt
for i in 1 2; do
timeout -k 10 300 python3 bench.py --model bert_base --steps 30 > $O/bert128_$i.txt 2>&1 || { tail -20 $O/bert128_$i.txt; exit 1; }
tail -1 $O/bert128_$i.txt | cut -c1-160
done
