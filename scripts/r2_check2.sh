#!/bin/bash
# Export / release / incremental / parity tests, then the library A/B on G3 and G2.
set -o pipefail
TAG=${1:-check}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_export.py tests/test_gpu_incremental.py tests/test_gpu_parity.py tests/test_gpu_workloads.py > $OUT/gpu.log 2>&1
rc=$?; tail -3 $OUT/gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/gpu.log | head -30; exit $rc; }
bash scripts/r2_lib_ab.sh $TAG/ab g3 "$@" && bash scripts/r2_lib_ab.sh $TAG/ab2 g2 "$@"
