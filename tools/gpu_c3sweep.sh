# usage: bash tools/gpu_c3sweep.sh TAG -- C3 parity with 2-chunk scatter, then launch-shape sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c3sweep}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BQGPU_PART_CHUNKS=2 timeout -k 10 400 python -u -m pytest tests -q -m gpu -rf -x -k "part or c3 or merge or limits" --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 tools/c3_sweep.py > $OUT/sweep.txt 2> $OUT/sweep.err || exit $?
cat $OUT/sweep.txt
