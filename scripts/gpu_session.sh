#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel stats.  Every GPU step has its
# own time limit and the chain stops at the first failure.  Usage: scripts/gpu_session.sh TAG [bench args]
set -o pipefail
TAG=${1:-run}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests -q -m gpu -x > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --verbose "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 "$@" > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find $OUT/prof -name "*kernel_stats.csv" -exec head -20 {} \;
exit $rc
