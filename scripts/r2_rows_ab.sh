#!/bin/bash
# Link-row sort check: export tests, then the wave sort vs the workgroup sort on G3 / G5.
set -o pipefail
TAG=${1:-rowsab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_export.py > $OUT/gpu.log 2>&1
rc=$?; tail -2 $OUT/gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/gpu.log | head -30; exit $rc; }
bash scripts/r2_cfg_ab.sh $TAG/ab g3 "distel_amd/lib/libel_gpu.so" "distel_amd/lib/libel_gpu.so EL_ROWS_NO_WAVE=1" && bash scripts/r2_cfg_ab.sh $TAG/ab5 g5 "distel_amd/lib/libel_gpu.so" "distel_amd/lib/libel_gpu.so EL_ROWS_NO_WAVE=1"
