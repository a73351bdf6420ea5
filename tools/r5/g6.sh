set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fp32_gpu.py tests/test_production_shapes_gpu.py > gpurun_out/r5_buf_tests.txt 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python -u bench.py --reference-config off > gpurun_out/r5_buf_bench.txt 2> gpurun_out/r5_buf_bench.err &&
timeout -k 10 600 python -u tools/tile_sweep.py > gpurun_out/r5_buf_tile_sweep.jsonl 2> gpurun_out/r5_buf_tile_sweep.err
echo "rc=$?"
