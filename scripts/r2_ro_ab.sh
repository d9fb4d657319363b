#!/bin/bash
# Read-out kernel check: export tests, then A/B of read-out variants on G3 (two in flight and serial).
set -o pipefail
TAG=${1:-roab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_export.py > $OUT/gpu.log 2>&1
rc=$?; tail -2 $OUT/gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/gpu.log | head -30; exit $rc; }
bash scripts/r2_cfg_ab.sh $TAG/ab g3 "distel_amd/lib/libel_gpu.so" "distel_amd/lib/libel_gpu.so EL_READOUT_WG=1" "distel_amd/lib/libel_gpu.so EL_READOUT_BLOCKS=256" "distel_amd/lib/libel_gpu.so EL_READOUT_BLOCKS=512"
