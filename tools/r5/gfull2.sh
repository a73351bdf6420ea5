# full GPU suite (no -x: every failure listed), smoke, default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 1000 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > $O/r5_gpu_full2.txt 2>&1
echo "full rc=$?"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r5_smoke2.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/r5_bench_default3.txt 2>&1 || exit 1
echo done
