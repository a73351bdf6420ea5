#!/bin/bash
# overlap GPU test; deterministic vs default same-box A/B on the current tree
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3u
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 300 python3 -u -m pytest -q -x --timeout 250 --timeout-method thread tests/test_ddp_gpu.py -k overlaps > $O/ovl_test.txt 2>&1 || { tail -30 $O/ovl_test.txt; exit 1; }
tail -1 $O/ovl_test.txt
for i in 1 2; do
  for d in 0 1; do
    timeout -k 10 300 python3 bench.py --steps 30 --deterministic $d > $O/b_d${d}_$i.txt 2>&1 || { tail -20 $O/b_d${d}_$i.txt; exit 1; }
    echo "det=$d $(tail -1 $O/b_d${d}_$i.txt | cut -c60-130)"
  done
done
