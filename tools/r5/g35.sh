# single-stage main loop with the next k-step's LDS-DMA under this k-step's MFMAs: tests + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_production_shapes_gpu.py tests/test_determinism_gpu.py tests/test_model_gpu.py > $O/r5_early_tests.txt 2>&1 || exit 1
S="fwd:256,56,64,64,3,1,1:9 fwd:256,28,128,128,3,1,1:1 fwd:256,56,64,256,1,1,0:9 fwd:256,56,256,64,1,1,0:9 dgrad:256,56,64,64,3,1,1:9 wgrad:256,56,64,256,1,1,0:9"
rm -f $O/r5_early_ops.jsonl
timeout -k 10 200 python -u tools/r5/conv_time.py early $S >> $O/r5_early_ops.jsonl || exit 1
ALT=/tmp/alt_loop3
rm -rf $ALT && mkdir -p $ALT && cp -r bench.py kubeflow-v2-distributed-pytorch_amd tools $ALT/ && ln -s kubeflow-v2-distributed-pytorch_amd $ALT/mipipe
cp tools/r5/alt/loop3/_C*.so $ALT/kubeflow-v2-distributed-pytorch_amd/
(cd $ALT && timeout -k 10 200 python -u tools/r5/conv_time.py loop3 $S >> $O/r5_early_ops.jsonl) || exit 1
rm -f $O/r5_early_ab.txt
bash tools/r5/ab_run.sh loop3 3 $O/r5_early_ab.txt --steps 30 --warmup 10 --reference-config off --time-deterministic off || exit 1
echo done
