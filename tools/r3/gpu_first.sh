#!/bin/bash
# Round 3, first GPU call: headline bench with clock samples, comm/compute overlap probe
# (eager and hipGraph replay), step-level force-reduce A/B, then the full GPU suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 300 python3 bench.py > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
tail -1 $O/bench.txt
timeout -k 10 240 python3 tools/r3/overlap_probe.py > $O/overlap_probe.txt 2>&1 || { tail -20 $O/overlap_probe.txt; exit 1; }
cat $O/overlap_probe.txt
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29511 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0
for g in on off; do
  timeout -k 10 240 python3 bench.py --force-reduce --graph $g --steps 30 --warmup 5 > $O/bench_fr_$g.txt 2>&1 || { tail -20 $O/bench_fr_$g.txt; exit 1; }
  tail -1 $O/bench_fr_$g.txt | cut -c1-400
done
unset MASTER_ADDR MASTER_PORT WORLD_SIZE RANK LOCAL_RANK
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
