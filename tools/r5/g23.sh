# MFMA BatchNorm statistics in the conv forward epilogue: tests, single-op times, same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_production_shapes_gpu.py tests/test_determinism_gpu.py tests/test_model_gpu.py > $O/r5_mstats_tests.txt 2>&1 || exit 1
ALT=/tmp/alt_valustats
rm -rf $ALT && mkdir -p $ALT && cp -r bench.py kubeflow-v2-distributed-pytorch_amd tools $ALT/ && ln -s kubeflow-v2-distributed-pytorch_amd $ALT/mipipe
cp tools/r5/alt/valustats/_C*.so $ALT/kubeflow-v2-distributed-pytorch_amd/
S="fwd:256,56,64,64,3,1,1:9 fwd:256,28,128,128,3,1,1:1 fwd:256,14,256,256,3,1,1:11 fwd:256,56,64,256,1,1,0:9 fwd:256,56,256,64,1,1,0:9 fwd:256,28,128,512,1,1,0:1 fwd:256,14,256,1024,1,1,0:1 fwd:256,7,512,2048,1,1,0:1"
rm -f $O/r5_mstats_ops.jsonl
timeout -k 10 200 python -u tools/r5/conv_time.py mfma $S >> $O/r5_mstats_ops.jsonl || exit 1
(cd $ALT && timeout -k 10 200 python -u tools/r5/conv_time.py valu $S >> $O/r5_mstats_ops.jsonl) || exit 1
rm -f $O/r5_mstats_ab.txt
bash tools/r5/ab_run.sh valustats 3 $O/r5_mstats_ab.txt --steps 30 --warmup 10 --reference-config off --time-deterministic off || exit 1
echo done
