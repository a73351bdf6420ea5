#!/bin/bash
# wide wave-tile configs 11 / 12: correctness of every config, per-shape tuning, bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "every_tile_config or every_plan or addend_epilogue" > $O/j_tests.txt 2>&1 || { tail -30 $O/j_tests.txt; exit 1; }
tail -2 $O/j_tests.txt
timeout -k 10 600 python3 tools/r2/tune_dump.py > $O/j_tune_dump.txt 2>&1 || { tail -20 $O/j_tune_dump.txt; exit 1; }
grep -E "^\[mipipe tune\] (fwd|dgrad)" $O/j_tune_dump.txt | awk '{print $3, $4, $5}' > $O/j_picks.txt
cat $O/j_picks.txt | head -60
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 30 > $O/j_new_$i.txt 2>&1 || { tail -20 $O/j_new_$i.txt; exit 1; }
  tail -1 $O/j_new_$i.txt | cut -c1-110
  MIPIPE_CONV_TILES=11 timeout -k 10 300 python3 bench.py --steps 30 > $O/j_old_$i.txt 2>&1 || { tail -20 $O/j_old_$i.txt; exit 1; }
  tail -1 $O/j_old_$i.txt | cut -c1-110
done
