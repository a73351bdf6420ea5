set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "embedding" > gpurun_out/r5_emb_tests.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_attention_gpu.py tests/test_ddp_gpu.py > gpurun_out/r5_bert_ddp_tests.txt 2>&1 &&
MASTER_ADDR=127.0.0.1 MASTER_PORT=29511 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 timeout -k 10 300 python -u bench.py --model bert_base --seq 128 --force-reduce --comm-dtype bf16 > gpurun_out/r5_bert_fr.txt 2> gpurun_out/r5_bert_fr.err &&
timeout -k 10 300 python -u bench.py --model bert_base --seq 128 > gpurun_out/r5_bert.txt 2> gpurun_out/r5_bert.err
echo "rc=$?"
