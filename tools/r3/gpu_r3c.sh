#!/bin/bash
# new GPU tests (reference invocation, BERT graph, dropout seeds, det+benchmark), reference pipeline
# on the GPU, DDP eager overlap with/without the high-priority RCCL stream, BERT graphed bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_task_gpu.py tests/test_attention_gpu.py tests/test_ddp_gpu.py tests/test_determinism_gpu.py tests/test_model_gpu.py > $O/c_tests.txt 2>&1 || { tail -60 $O/c_tests.txt; exit 1; }
tail -3 $O/c_tests.txt
export MIPIPE_GCS_ROOT=$O/gcs_root
timeout -k 10 600 python3 examples/reference_pipeline.py --replicas 1 --gpus-per-replica 1 --spec $O/ref_dag.json --extra-args '["--batch_size=256","--train-samples=4096","--test-samples=1024","--eval-every=1"]' > $O/ref_pipeline_gpu.txt 2>&1 || { tail -40 $O/ref_pipeline_gpu.txt; exit 1; }
tail -5 $O/ref_pipeline_gpu.txt
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29511 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0
for hp in 1 0; do
  TORCH_NCCL_HIGH_PRIORITY=$hp timeout -k 10 300 python3 bench.py --force-reduce --graph off --steps 30 > $O/fr_eager_hp$hp.txt 2>&1 || { tail -20 $O/fr_eager_hp$hp.txt; exit 1; }
  tail -1 $O/fr_eager_hp$hp.txt | cut -c1-250
done
timeout -k 10 300 python3 bench.py --graph off --steps 30 > $O/nofr_eager.txt 2>&1 || { tail -20 $O/nofr_eager.txt; exit 1; }
tail -1 $O/nofr_eager.txt | cut -c1-250
timeout -k 10 300 python3 bench.py --model bert_base --seq 128 --force-reduce --steps 30 > $O/bert_graph_fr.txt 2>&1 || { tail -20 $O/bert_graph_fr.txt; exit 1; }
tail -1 $O/bert_graph_fr.txt | cut -c1-600
unset MASTER_ADDR MASTER_PORT WORLD_SIZE RANK LOCAL_RANK
timeout -k 10 300 python3 bench.py --model bert_base --seq 128 --steps 30 > $O/bert_graph.txt 2>&1 || { tail -20 $O/bert_graph.txt; exit 1; }
tail -1 $O/bert_graph.txt | cut -c1-300
timeout -k 10 300 python3 bench.py --model bert_base --seq 128 --steps 30 --graph off > $O/bert_eager.txt 2>&1 || { tail -20 $O/bert_eager.txt; exit 1; }
tail -1 $O/bert_eager.txt | cut -c1-300
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29512 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_ddp -o run -- python3 $R/bench.py --force-reduce --graph off --steps 3 --warmup 2 > $O/prof_ddp.txt 2>&1 || { tail -20 $O/prof_ddp.txt; exit 1; }
cd $R
T=$(ls $O/prof_ddp/*/run_kernel_trace.csv $O/prof_ddp/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 tools/overlap_report.py $T > $O/ddp_overlap_eager_hp.txt
tail -3 $O/ddp_overlap_eager_hp.txt
