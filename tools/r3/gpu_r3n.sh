#!/bin/bash
# experiment: conv weight-grads on a side stream (MIPIPE_SIDE_WGRAD=1) vs on the compute stream
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3n
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
for i in 1 2; do
  for sw in 1 0; do
    MIPIPE_SIDE_WGRAD=$sw timeout -k 10 300 python3 bench.py --steps 30 > $O/g_$sw_$i.txt 2>&1 || { tail -20 $O/g_$sw_$i.txt; exit 1; }
    echo "graph side=$sw $(tail -1 $O/g_$sw_$i.txt | cut -c1-150)"
  done
done
for sw in 1 0; do
  MIPIPE_SIDE_WGRAD=$sw timeout -k 10 300 python3 bench.py --steps 20 --graph off > $O/e_$sw.txt 2>&1 || { tail -20 $O/e_$sw.txt; exit 1; }
  echo "eager side=$sw $(tail -1 $O/e_$sw.txt | cut -c1-150)"
  MIPIPE_SIDE_WGRAD=$sw timeout -k 10 300 python3 bench.py --steps 10 --deterministic 1 > $O/d_$sw.txt 2>&1 || { tail -20 $O/d_$sw.txt; exit 1; }
  echo "det side=$sw $(tail -1 $O/d_$sw.txt | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], repr(j["final_loss"]))')"
done
