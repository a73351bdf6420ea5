#!/bin/bash
# final tree: smoke + full pytest -m gpu (no benches)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3zj
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
