set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_determinism_gpu.py tests/test_fp32_gpu.py tests/test_tap_crop.py tests/test_model_gpu.py > $O/r5_det_direct_tests.txt 2>&1 || { echo tests failed; tail -20 $O/r5_det_direct_tests.txt; exit 1; }
timeout -k 10 300 python -u bench.py > $O/r5_bench_default2.txt 2> $O/r5_bench_default2.err || exit 1
echo done
