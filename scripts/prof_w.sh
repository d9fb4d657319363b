#!/bin/bash
# rocprofv3 kernel trace of one workload's bench (scripts/prof_w.sh TAG WORKLOAD)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --workload $2 --no-cpu --no-profile --steps 2 --warmup 1 > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
