set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fp32_gpu.py tests/test_production_shapes_gpu.py tests/test_determinism_gpu.py > $O/r5_epi_tests.txt 2>&1 || { echo "tests failed"; exit 1; }
rm -f $O/r5_ab_epi.txt $O/r5_ab_epi_bert.txt
bash tools/r5/ab_run.sh nobuf 3 $O/r5_ab_epi.txt --reference-config off --time-deterministic off || exit 1
bash tools/r5/ab_run.sh nobuf 2 $O/r5_ab_epi_bert.txt --model bert_base --seq 128 || exit 1
bash tools/r4/pmc_conv.sh r5epi_l3c2_fwd 256 14 256 256 3 1 1 fwd -1 > /dev/null 2>&1 || exit 1
bash tools/r4/pmc_gemm.sh r5epi_qkv 4096,2304,768,1,1,0 -1 > /dev/null 2>&1 || exit 1
echo done
