#!/bin/bash
# round 6 H: the whole GPU suite + smoke at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6h}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -2 $OUT/smoke.txt
