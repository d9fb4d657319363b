#!/bin/bash
# One measurement session on the current source: whole GPU suite, the default bench line
# (G3 with copy-back, roofline, cpu_baseline), a rocprofv3 kernel-trace --stats run of the
# same bench, then the FETCH_SIZE / WRITE_SIZE PMC passes (separate runs, no tracing).
# Usage: scripts/r2_session.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-session}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > $OUT/gpu.log 2>&1
  rc=$?; tail -3 $OUT/gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/gpu.log | head -30; exit $rc; }
fi
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --no-cpu --no-profile --steps 5 --warmup 1 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $OUT/prof.log; exit 1; }
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --no-cpu --no-profile --steps 1 --warmup 0 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
