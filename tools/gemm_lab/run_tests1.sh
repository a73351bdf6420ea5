cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "every_plan or splitk_bf16 or addend_epilogue or every_tile_config or identity" > gpurun_out/t1.log 2>&1
rc=$?
tail -30 gpurun_out/t1.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_oneshot_gpu.py > gpurun_out/t2.log 2>&1
rc=$?
tail -30 gpurun_out/t2.log
exit $rc
