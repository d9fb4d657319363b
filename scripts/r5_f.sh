#!/bin/bash
# GPU session (scripts/r5_f.sh TAG VARIANT...): parity of the closure paths (KATs, cycles, fuzz,
# pinned digests incl. full G3), then scripts/r4_ab.sh's G3 A/B of the default build against the
# variants.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_workloads.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash scripts/r4_ab.sh "$@"
