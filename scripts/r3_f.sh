#!/bin/bash
# GPU session (scripts/r3_f.sh TAG [notests]): the GPU suite, the G3 bench line, a rocprofv3
# kernel trace of the same bench (stats summary printed).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
if [ "$2" != "notests" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/gpu.log 2>&1
  rc=$?; tail -3 $OUT/gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/gpu.log | head -20; exit $rc; }
fi
timeout -k 10 300 python bench.py --workload g3 --no-cpu --steps 5 --warmup 2 > $OUT/g3.json 2> $OUT/g3.err || { tail $OUT/g3.err; exit 1; }
cat $OUT/g3.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o g3 -- python $R/bench.py --workload g3 --no-cpu --no-profile --no-throughput2 --steps 3 --warmup 1 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
python3 $R/scripts/rpd_stats.py "$OUT/prof/**/*.db" | cut -c1-120 | head -25
