#!/bin/bash
# GPU session (scripts/r4_baseline.sh TAG): BASELINE.md §3 lines — bench.py on every workload at
# N = 1 (profiled roofline pass on), and the CPU oracle classifying each whole workload on one
# host core of the same box (oracle/cpu_baseline.py W 1.0 1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for w in g3 g1 g2 g5 g3x; do
  timeout -k 10 240 python bench.py --workload $w --no-cpu --steps 10 --warmup 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err \
    || { tail $OUT/bench_$w.err; exit 1; }
  echo "$w $(python -c "import json; d=json.load(open('$OUT/bench_$w.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])")"
done
for w in g1 g2 g5 g3 g3x; do
  timeout -k 10 200 python oracle/cpu_baseline.py $w 1.0 1 > $OUT/cpu_$w.json 2> $OUT/cpu_$w.err || { tail $OUT/cpu_$w.err; exit 1; }
  echo "cpu $w $(cat $OUT/cpu_$w.json | cut -c1-300)"
done
