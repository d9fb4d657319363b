#!/bin/bash
# Round-end measurement on the final source: whole GPU suite; the default bench line (G3, two in
# flight, roofline, cpu_baseline); G2 / G5 / G3X / serial-G3 lines; rocprofv3 kernel stats of the
# default bench and a serial kernel trace (per-superstep table); FETCH_SIZE / WRITE_SIZE passes.
# Usage: scripts/r2_final.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > $OUT/gpu.log 2>&1
  rc=$?; tail -3 $OUT/gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/gpu.log | head -30; exit $rc; }
fi
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --verbose > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
for cfg in "g2 2" "g5 2" "g3x 2" "g3 1" "g2 1"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --workload $1 --inflight $2 --no-cpu --no-profile --steps 20 --warmup 5 > $OUT/$1_$2.json 2> $OUT/$1_$2.err || { tail -5 $OUT/$1_$2.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$1_$2.json')); print('$1 inflight $2', d['ms_per_step'], 'ms', 'sat', d['saturate_ms'], 'lat', d['latency_ms'], 'copy', d['copyback_ms'], round(d['value']/1e9,3), 'G/s')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --no-cpu --no-profile --steps 5 --warmup 1 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $OUT/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --inflight 1 --no-cpu --no-profile --steps 2 --warmup 1 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --inflight 1 --no-cpu --no-profile --steps 1 --warmup 0 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
