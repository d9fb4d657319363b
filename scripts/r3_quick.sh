#!/bin/bash
# Quick GPU check (scripts/r3_quick.sh TAG): parity suite, G3 bench line (no CPU leg), rocprofv3
# kernel trace of the same bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_export.py > $OUT/gpu.log 2>&1
rc=$?; tail -2 $OUT/gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/gpu.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --workload g3 --no-cpu --no-throughput2 --steps 5 --warmup 2 > $OUT/g3.json 2> $OUT/g3.err || { tail $OUT/g3.err; exit 1; }
cat $OUT/g3.json
timeout -k 10 300 python bench.py --workload g3 --no-cpu --no-throughput2 --copyback rows --steps 5 --warmup 2 > $OUT/g3rows.json 2>> $OUT/g3.err && cat $OUT/g3rows.json || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o g3 -- python $R/bench.py --workload g3 --no-cpu --no-profile --no-throughput2 --steps 3 --warmup 1 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
python3 $R/scripts/rpd_stats.py "$OUT/prof/**/*.db" | cut -c1-120 | head -25
