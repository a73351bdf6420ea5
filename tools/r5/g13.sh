set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_tap_crop.py tests/test_fp32_gpu.py -k "crop or resnet18" > $O/r5_crop_tests.txt 2>&1 || { echo tests failed; tail -30 $O/r5_crop_tests.txt; exit 1; }
REF="--model resnet18 --res 32 --batch 1024 --dtype fp32 --deterministic 1 --reference-config off --time-deterministic off"
timeout -k 10 300 python -u bench.py $REF --tune 2 --save-tune $O/r5_r18_f32_table.json > $O/r5_tablegen.txt 2>&1 || exit 1
rm -f $O/r5_crop_ab.txt
bash tools/r5/env_ab.sh $O/r5_crop_ab.txt 2 MIPIPE_TAP_CROP=0 MIPIPE_TAP_CROP=1 -- $REF || exit 1
bash tools/r5/env_ab.sh $O/r5_crop_ab.txt 1 MIPIPE_TAP_CROP=1 MIPIPE_TUNE_TABLE=$O/r5_r18_f32_table.json -- $REF || exit 1
bash tools/r5/env_ab.sh $O/r5_crop_ab_bf16.txt 1 MIPIPE_TAP_CROP=0 MIPIPE_TAP_CROP=1 -- --model resnet18 --res 32 --batch 1024 --reference-config off --time-deterministic off || exit 1
echo done
