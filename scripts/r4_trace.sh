#!/bin/bash
# GPU session (scripts/r4_trace.sh TAG): rocprofv3 kernel traces of the timed G3 bench, with the
# process bound to the GPU's NUMA node (default) and unbound (EL_NUMA_BIND=0), beside an untraced
# run of each: how far tracing dilates the step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
B="bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3"
for v in 0 1; do
  EL_NUMA_BIND=$v timeout -k 10 200 python $B > $OUT/u_$v.json 2> $OUT/u_$v.err || { tail $OUT/u_$v.err; exit 1; }
  (cd /tmp && EL_NUMA_BIND=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr$v -o tr -- python3 $R/$B > $OUT/tr$v.json 2> $OUT/tr$v.err) || { tail $OUT/tr$v.err; exit 1; }
  echo "bind=$v untraced $(python -c "import json; d=json.load(open('$OUT/u_$v.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'])") traced $(python -c "import json; d=json.loads(open('$OUT/tr$v.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'])")"
  python3 scripts/rpd_stats.py $OUT/tr$v/tr_results.db > $OUT/tr${v}_stats.csv && head -4 $OUT/tr${v}_stats.csv
done
