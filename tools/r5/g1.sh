set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -s \
  tests/test_fp32_gpu.py -k "resnet18_cifar" > gpurun_out/r5_fp32_model.txt 2>&1 &&
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "every_plan or every_tile or workspace_plans" > gpurun_out/r5_every_plan.txt 2>&1 ;
echo "every_plan rc=$?" ;
timeout -k 10 300 python -u bench.py > gpurun_out/r5_bench1.txt 2> gpurun_out/r5_bench1.err &&
timeout -k 10 300 python -u bench.py --impl stock --model resnet18 --res 32 --batch 1024 --dtype fp32 --reference-config off > gpurun_out/r5_stock_r18fp32.txt 2>&1
echo "done rc=$?"
