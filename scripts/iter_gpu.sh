#!/bin/bash
# Iteration check (scripts/iter_gpu.sh TAG): GPU parity suite, G2/G3 bench lines, kernel traces
# of G2 and G3 (per-superstep tables via scripts/steps.py).
set -o pipefail
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
cd /tmp && export TMPDIR=/tmp
for w in g2 g3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_$w -o run -- python3 $R/bench.py --workload $w --no-cpu --no-profile --steps 2 --warmup 1 > $OUT/tr_$w.log 2>&1 || exit 1
done
echo traced
