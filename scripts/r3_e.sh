#!/bin/bash
# GPU session (scripts/r3_e.sh TAG): runtime log of the streamed copies, the GPU suite, the G3
# bench line, a rocprofv3 kernel trace of the same bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
AMD_LOG_LEVEL=4 timeout -k 10 120 python scripts/copylog.py > $OUT/copylog.txt 2>&1 || { tail -5 $OUT/copylog.txt; exit 1; }
grep -iE "copy|blit|sdma" $OUT/copylog.txt | grep -v "^$" | tail -40 > $OUT/copylog_grep.txt; wc -l $OUT/copylog.txt; tail -3 $OUT/copylog.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/gpu.log 2>&1
rc=$?; tail -3 $OUT/gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/gpu.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --workload g3 --no-cpu --steps 5 --warmup 2 > $OUT/g3.json 2> $OUT/g3.err || { tail $OUT/g3.err; exit 1; }
cat $OUT/g3.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o g3 -- python $R/bench.py --workload g3 --no-cpu --no-profile --no-throughput2 --steps 3 --warmup 1 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
python3 $R/scripts/rpd_stats.py "$OUT/prof/**/*.db" | cut -c1-120 | head -25
# FETCH_SIZE / WRITE_SIZE calibration of the saturation's access patterns (scripts/micro/pmc_cal.hip)
timeout -k 10 60 $R/scripts/micro/pmc_cal > $OUT/cal.txt 2>&1 || { cat $OUT/cal.txt; exit 1; }
cat $OUT/cal.txt
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c1 -o c -- $R/scripts/micro/pmc_cal > $OUT/c1.log 2>&1 || { tail -3 $OUT/c1.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c2 -o c -- $R/scripts/micro/pmc_cal > $OUT/c2.log 2>&1 || { tail -3 $OUT/c2.log; exit 1; }
python3 $R/scripts/pmc_cal_summary.py $OUT $OUT/pmc_calibration.json
