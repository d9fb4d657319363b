#!/bin/bash
# Diagnostic: rocprofv3 kernel trace of the G2 bench with the commit roles split in two launches.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export EL_SPLIT_COMMIT=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --no-cpu --no-profile --steps 2 --warmup 1 > $OUT/prof.log 2>&1
echo "rocprof rc=$?"
