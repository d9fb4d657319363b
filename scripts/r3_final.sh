#!/bin/bash
# Round-3 final GPU session (scripts/r3_final.sh TAG): the whole GPU suite, the default bench line
# (with cpu_baseline), a rocprofv3 kernel trace + stats of the timed bench, lines for G2 / G5 /
# G3X, and one full-G3 classification of the CPU oracle on one host core.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/gpu.log 2>&1
rc=$?; tail -2 $OUT/gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/gpu.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py > $OUT/final.json 2> $OUT/final.err || { tail $OUT/final.err; exit 1; }
cat $OUT/final.json
for w in g2 g5 g3x; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu --no-throughput2 --steps 10 --warmup 3 > $OUT/$w.json 2>> $OUT/lines.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], d['derived_axioms'], d['init_ms'], d['saturate_ms'])" $OUT/$w.json $w
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o g3 -- python $R/bench.py --workload g3 --no-cpu --no-profile --no-throughput2 --steps 3 --warmup 1 > $OUT/prof.log 2>&1) || { tail $OUT/prof.log; exit 1; }
python3 scripts/rpd_stats.py "$OUT/prof/**/*.db" --csv $OUT/kernel_trace_stats.csv | head -12
timeout -k 10 600 python oracle/cpu_baseline.py g3 1.0 1 > $OUT/cpu_full_g3.json 2> $OUT/cpu_full.err
cat $OUT/cpu_full_g3.json
