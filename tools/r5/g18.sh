set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_tap_crop.py tests/test_fp32_gpu.py tests/test_model_gpu.py tests/test_determinism_gpu.py > $O/r5_flat_tests.txt 2>&1 || { echo tests failed; tail -30 $O/r5_flat_tests.txt; exit 1; }
rm -f $O/r5_flat_ab.txt
REF="--model resnet18 --res 32 --batch 1024 --dtype fp32 --deterministic 1 --reference-config off --time-deterministic off"
bash tools/r5/env_ab.sh $O/r5_flat_ab.txt 2 MIPIPE_TAP_CROP=0 MIPIPE_TAP_CROP=1 -- $REF || exit 1
echo done
