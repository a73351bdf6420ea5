#!/bin/bash
# Round-end evidence: full GPU suite (one process), smoke, 1-GPU headline bench, deterministic
# bench, ResNet-50 eager per-call profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/final_tests.txt 2>&1 || { tail -40 $O/final_tests.txt; exit 1; }
tail -1 $O/final_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/final_smoke.txt 2>&1 || { tail -20 $O/final_smoke.txt; exit 1; }
tail -1 $O/final_smoke.txt
timeout -k 10 300 python3 $R/bench.py > $O/final_bench.txt 2>&1 || { tail -20 $O/final_bench.txt; exit 1; }
tail -1 $O/final_bench.txt | cut -c1-200
timeout -k 10 300 python3 $R/bench.py --deterministic 1 > $O/final_bench_det.txt 2>&1 || { tail -20 $O/final_bench_det.txt; exit 1; }
tail -1 $O/final_bench_det.txt | cut -c1-200
bash $R/tools/r2/gpu_percall.sh
