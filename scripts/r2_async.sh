#!/bin/bash
# Async copy-back check: the async tests, then the bench with 2 engines in flight vs serial.
set -o pipefail
TAG=${1:-async}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_export.py -k "async or release" > $OUT/gpu.log 2>&1
rc=$?; tail -3 $OUT/gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/gpu.log | head -30; exit $rc; }
for cfg in "g3 2" "g3 1" "g2 2" "g2 1" "g5 2"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --workload $1 --inflight $2 --no-cpu --no-profile --steps 20 --warmup 5 > $OUT/$1_$2.json 2> $OUT/$1_$2.err || { tail -5 $OUT/$1_$2.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$1_$2.json')); print('$1 inflight $2', d['ms_per_step'], 'ms', 'sat', d['saturate_ms'], 'lat', d['latency_ms'], 'copy', d['copyback_ms'], round(d['value']/1e9,3), 'G/s')"
done
