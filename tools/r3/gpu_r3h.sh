#!/bin/bash
# deterministic-mode tune table: build it (det kernels timed), then det-with-table vs default A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 400 python3 bench.py --deterministic 1 --tune 2 --save-tune $O/tune_det_r50.json --steps 10 > $O/h_tune.txt 2>&1 || { tail -20 $O/h_tune.txt; exit 1; }
tail -1 $O/h_tune.txt | cut -c1-200
python3 -c "import json; print(len(json.load(open('$O/tune_det_r50.json'))), 'entries')"
cp $O/tune_det_r50.json kubeflow-v2-distributed-pytorch_amd/ops/tune_tables/gfx950_resnet50_b256.json
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --deterministic 1 --steps 30 > $O/h_det_$i.txt 2>&1 || { tail -20 $O/h_det_$i.txt; exit 1; }
  tail -1 $O/h_det_$i.txt | cut -c1-120
  timeout -k 10 300 python3 bench.py --steps 30 > $O/h_def_$i.txt 2>&1 || { tail -20 $O/h_def_$i.txt; exit 1; }
  tail -1 $O/h_def_$i.txt | cut -c1-120
done
