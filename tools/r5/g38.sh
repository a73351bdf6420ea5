# fp32 epilogue staged in two row passes when it would exceed the main loop's LDS (more blocks per
# CU for single-stage weight-grads) + early DMA for the GEMM kernels: tests + A/B (ResNet-50, BERT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_production_shapes_gpu.py tests/test_determinism_gpu.py tests/test_model_gpu.py tests/test_attention_gpu.py > $O/r5_f32p_tests.txt 2>&1 || exit 1
rm -f $O/r5_f32p_ab.txt $O/r5_f32p_ab_bert.txt
bash tools/r5/ab_run.sh old3 3 $O/r5_f32p_ab.txt --steps 30 --warmup 10 --reference-config off --time-deterministic off || exit 1
bash tools/r5/ab_run.sh old3 2 $O/r5_f32p_ab_bert.txt --model bert_base --seq 128 --steps 30 --warmup 10 --reference-config off --time-deterministic off || exit 1
echo done
