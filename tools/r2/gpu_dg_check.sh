set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/dg
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_shapes_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/dg/kernels.txt 2>&1; echo "kernels rc=$?"; tail -15 gpurun_out/dg/kernels.txt | grep -v "^$"
MIPIPE_DGRAD_FWD=0 timeout -k 10 200 python -u -m pytest tests/test_ddp_gpu.py -q -k graphed --timeout 150 --timeout-method thread > gpurun_out/dg/ddp0.txt 2>&1; echo "ddp fwd=0 rc=$?"; grep "^E  .*AssertionError\|passed\|failed" gpurun_out/dg/ddp0.txt | head -3
MIPIPE_DGRAD_FWD=1 timeout -k 10 200 python -u -m pytest tests/test_ddp_gpu.py -q -k graphed --timeout 150 --timeout-method thread > gpurun_out/dg/ddp1.txt 2>&1; echo "ddp fwd=1 rc=$?"; grep "^E  .*AssertionError\|passed\|failed" gpurun_out/dg/ddp1.txt | head -3
