#!/bin/bash
# rocprofv3 kernel + memory-copy trace of a short bench run (no counters).  Usage: scripts/r2_prof.sh TAG WORKLOAD
set -o pipefail
TAG=${1:-prof}; W=${2:-g3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --workload $W --no-cpu --no-profile --steps 3 --warmup 1 > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 $OUT/prof.log
find $OUT/prof -name "*stats.csv" | while read f; do echo "== $f"; head -30 "$f"; done
exit $rc
