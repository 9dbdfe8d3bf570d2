#!/bin/bash
# round 6 AO: the whole GPU suite and smoke at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r6ao}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 500 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
