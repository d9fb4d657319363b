#!/bin/bash
# Whole GPU suite (one process), then the G3 / G5 / G3X bench lines.  Usage: scripts/r2_full.sh TAG
set -o pipefail
TAG=${1:-full}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > $OUT/gpu.log 2>&1
rc=$?; tail -3 $OUT/gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/gpu.log | head -30; exit $rc; }
for w in g3 g5 g3x g2; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu --no-profile --steps 10 --warmup 3 > $OUT/$w.json 2> $OUT/$w.err || { tail -5 $OUT/$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$w.json')); print('$w', d['ms_per_step'], 'ms', 'sat', d['saturate_ms'], 'copy', d['copyback_ms'], d['copyback_gbs'], 'GB/s', round(d['value']/1e9,3), 'G/s')"
done
