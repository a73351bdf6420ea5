#!/bin/bash
# wgrad3x3 4- vs 8-wave A/B (+ off), kernel timing; re-capture pipeline log and DDP overlap report
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3f
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad3x3_gpu.py > $O/w3_tests8.txt 2>&1 || { tail -40 $O/w3_tests8.txt; exit 1; }
tail -1 $O/w3_tests8.txt
MIPIPE_WGRAD3_WAVES=4 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad3x3_gpu.py > $O/w3_tests4.txt 2>&1 || { tail -40 $O/w3_tests4.txt; exit 1; }
tail -1 $O/w3_tests4.txt
for i in 1 2; do
  for v in 8 4; do
    MIPIPE_WGRAD3_WAVES=$v timeout -k 10 300 python3 bench.py --steps 30 > $O/b_w$v_$i.txt 2>&1 || { tail -20 $O/b_w$v_$i.txt; exit 1; }
    echo "waves=$v $(tail -1 $O/b_w$v_$i.txt | cut -c1-150)"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in 8 4; do
  MIPIPE_WGRAD3_WAVES=$v timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_w$v -o run -- python3 $R/bench.py --steps 3 --warmup 4 --graph off > $O/prof_w$v.txt 2>&1 || { tail -20 $O/prof_w$v.txt; exit 1; }
  T=$(ls $O/prof_w$v/*/run_kernel_trace.csv $O/prof_w$v/run_kernel_trace.csv 2>/dev/null | head -n 1)
  python3 $R/tools/r2/per_call.py $T > $O/calls_w$v.txt
  python3 $R/tools/kernel_stats.py $T --step-marker sgd --last 3 --top 40 > $O/stats_w$v.txt
  rm -rf $O/prof_w$v
  echo "waves=$v"; grep -E "wgrad3x3|splitk" $O/calls_w$v.txt | awk '{print $2, $4, $NF}' | head -30
done
cd $R
export MIPIPE_GCS_ROOT=/tmp/gcs_root_r3f
timeout -k 10 600 python3 examples/reference_pipeline.py --replicas 1 --gpus-per-replica 1 --spec $O/ref_dag.json --extra-args '["--batch_size=256","--train-samples=4096","--test-samples=1024","--eval-every=1"]' > $O/ref_pipeline_gpu.txt 2>&1 || { tail -40 $O/ref_pipeline_gpu.txt; exit 1; }
cp $(ls /tmp/gcs_root_r3f/test-pkl/pipeline_root/*/run.json | head -1) $O/ref_pipeline_run.json
cp $(ls /tmp/gcs_root_r3f/test-pkl/jobs/*/logs/rank0.log | head -1) $O/ref_pipeline_rank0.log
tail -2 $O/ref_pipeline_gpu.txt
unset MIPIPE_GCS_ROOT
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29512 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_ddp -o run -- python3 $R/bench.py --force-reduce --graph off --steps 3 --warmup 2 > $O/prof_ddp.txt 2>&1 || { tail -20 $O/prof_ddp.txt; exit 1; }
T=$(ls $O/prof_ddp/*/run_kernel_trace.csv $O/prof_ddp/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 $R/tools/overlap_report.py $T > $O/ddp_overlap_eager_hp.txt
rm -rf $O/prof_ddp
tail -2 $O/ddp_overlap_eager_hp.txt
du -sh $O
