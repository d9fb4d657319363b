#!/bin/bash
# Round-2 GPU check: export/copy-back parity, then G2 / G3 bench lines (copy-back in the step).
# Usage: scripts/r2_gpu.sh TAG [pytest selection]
set -o pipefail
TAG=${1:-r2}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
SEL=${@:-tests/test_gpu_export.py}
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu $SEL > $OUT/gpu.log 2>&1
rc=$?; tail -3 $OUT/gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/gpu.log | head -30; exit $rc; }
for w in g2 g3; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu --no-profile --steps 10 --warmup 3 > $OUT/$w.json 2> $OUT/$w.err || { tail -5 $OUT/$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$w.json')); print('$w', d['ms_per_step'], 'ms', 'sat', d['saturate_ms'], 'copy', d['copyback_ms'], d['copyback_gbs'], 'GB/s', round(d['value']/1e9,3), 'G/s')"
done
