#!/bin/bash
# GPU session (scripts/r6_tests.sh TAG [pytest -k expr]): the -m gpu suite (or a -k subset) with a
# hang guard per test.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $OUT/t.log 2>&1
rc=$?; tail -3 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
