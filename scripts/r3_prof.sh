#!/bin/bash
# GPU timeline check (scripts/r3_prof.sh TAG [bench args...]): environment, verbose G3 bench line,
# rocprofv3 kernel trace of the same bench (DB under gpurun_out/TAG/prof).
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; shift
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
env | grep -iE "sdma|^hip|^hsa|^gpu_|^roc" > $OUT/env.txt
timeout -k 10 300 python bench.py --workload g3 --no-cpu --no-throughput2 --verbose --steps 5 --warmup 2 "$@" > $OUT/g3.json 2> $OUT/g3.err || { tail $OUT/g3.err; exit 1; }
cat $OUT/g3.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o g3 -- python $R/bench.py --workload g3 --no-cpu --no-profile --no-throughput2 --steps 3 --warmup 1 "$@" > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
python3 $R/scripts/rpd_stats.py "$OUT/prof/**/*.db" | cut -c1-120 | head -25
