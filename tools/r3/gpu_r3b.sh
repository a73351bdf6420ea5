#!/bin/bash
# overlap experiments + eager per-call profile + deterministic tune table and det/default A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
bash tools/r3/gpu_overlap.sh || exit 1
# deterministic tune table: time the candidates (forced) during warm-up, save
timeout -k 10 400 python3 bench.py --deterministic 1 --tune 2 --save-tune $O/tune_det_r50.json --steps 5 --warmup 3 > $O/tune_det.txt 2>&1 || { tail -20 $O/tune_det.txt; exit 1; }
tail -1 $O/tune_det.txt | cut -c1-300
cp $O/tune_det_r50.json mipipe/ops/tune_tables/gfx950_resnet50_b256.json
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 30 > $O/ab_def_$i.txt 2>&1 || { tail -20 $O/ab_def_$i.txt; exit 1; }
  tail -1 $O/ab_def_$i.txt | cut -c1-200
  timeout -k 10 300 python3 bench.py --steps 30 --deterministic 1 > $O/ab_det_$i.txt 2>&1 || { tail -20 $O/ab_det_$i.txt; exit 1; }
  tail -1 $O/ab_det_$i.txt | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_pc -o run -- python3 $R/bench.py --steps 3 --warmup 4 --graph off > $O/pc_prof.txt 2>&1 || { tail -20 $O/pc_prof.txt; exit 1; }
cd $R
T=$(ls $O/prof_pc/*/run_kernel_trace.csv $O/prof_pc/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/r2/per_call.py $T > $O/pc_calls.txt
python3 tools/kernel_stats.py $T --step-marker sgd --last 3 --top 40 > $O/pc_stats.txt
head -3 $O/pc_stats.txt
