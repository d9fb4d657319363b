#!/bin/bash
# Quick GPU check (scripts/quick_gpu.sh TAG): GPU parity suite, then G2/G3/G5 bench lines
# (no CPU leg, no profile) and G3 candidates per step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu.log 2>&1
rc=$?; tail -2 $OUT/gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/gpu.log | head -20; exit $rc; }
for w in g2 g3 g5; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu --no-profile --steps 5 --warmup 2 > $OUT/$w.json 2> $OUT/$w.err || exit 1
  echo "$w $(python -c "import json; d=json.load(open('$OUT/$w.json')); print(d['ms_per_step'], 'ms', d['supersteps'], 'steps', round(d['value']/1e9,3), 'G/s')")"
done
timeout -k 10 200 python scripts/cands.py g3 > $OUT/c3.log 2>&1 || exit 1
head -4 $OUT/c3.log
timeout -k 10 300 python scripts/trace_check.py g3 || exit 1
