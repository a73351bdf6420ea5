# branch-free FastDiv + fused data-grad BN-backward sums as Σg, Σg·y + stem counted waits:
# tests, then A/B vs the previous commit (old2) and vs the centered BN-backward sums (bnrc)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_production_shapes_gpu.py tests/test_determinism_gpu.py tests/test_model_gpu.py tests/test_fp32_gpu.py tests/test_stem_fused_gpu.py > $O/r5_bnr_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -q --timeout 250 --timeout-method thread tests/test_ddp_gpu.py -k overlaps_compute > $O/r5_overlap_test.txt 2>&1
rm -f $O/r5_bnr_ab.txt $O/r5_fd_ab.txt
bash tools/r5/ab_run.sh old2 3 $O/r5_fd_ab.txt --steps 30 --warmup 10 --reference-config off --time-deterministic off || exit 1
bash tools/r5/ab_run.sh bnrc 2 $O/r5_bnr_ab.txt --steps 30 --warmup 10 --reference-config off --time-deterministic off || exit 1
echo done
