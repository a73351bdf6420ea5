set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/dg
timeout -k 10 400 python -u -m pytest tests/test_determinism_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/dg/det.txt 2>&1; echo "det rc=$?"; grep "^E  .*Error\|passed\|failed" gpurun_out/dg/det.txt | head -5
for i in 1 2; do MIPIPE_DGRAD_FWD=0 timeout -k 10 200 python -u -m pytest tests/test_ddp_gpu.py -q -k graphed --timeout 150 --timeout-method thread -s > gpurun_out/dg/ddp0_$i.txt 2>&1; echo "ddp fwd=0 rc=$?"; grep "COS\|^E  .*AssertionError\|passed\|failed" gpurun_out/dg/ddp0_$i.txt | head -3; done
