#!/bin/bash
# rebuild the shipped deterministic-mode tile table on the current kernels; det vs default A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3w
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
MIPIPE_SHIPPED_TUNE=0 timeout -k 10 600 python3 bench.py --deterministic 1 --tune 2 --save-tune $O/det_table.json --steps 3 --warmup 3 > $O/make_table.txt 2>&1 || { tail -20 $O/make_table.txt; exit 1; }
tail -1 $O/make_table.txt | cut -c1-120
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 30 > $O/b_def_$i.txt 2>&1 || { tail -20 $O/b_def_$i.txt; exit 1; }
  echo "default $(tail -1 $O/b_def_$i.txt | cut -c60-120)"
  MIPIPE_TUNE_TABLE=$O/det_table.json timeout -k 10 300 python3 bench.py --steps 30 --deterministic 1 > $O/b_det_$i.txt 2>&1 || { tail -20 $O/b_det_$i.txt; exit 1; }
  echo "det new table $(tail -1 $O/b_det_$i.txt | cut -c60-120)"
done
timeout -k 10 300 python3 bench.py --steps 30 --deterministic 1 > $O/b_det_old.txt 2>&1 || { tail -20 $O/b_det_old.txt; exit 1; }
echo "det old shipped table $(tail -1 $O/b_det_old.txt | cut -c60-120)"
