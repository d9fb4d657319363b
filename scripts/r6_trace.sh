#!/bin/bash
# GPU session (scripts/r6_trace.sh TAG [workload]): rocprofv3 kernel trace (--stats) of the timed
# bench, its kernel table (rpd_stats.py) and per-superstep walls (steps.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
W=${2:-g3}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
B="bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3 --workload $W"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o tr -- python3 $R/$B > $OUT/tr.json 2> $OUT/tr.err) || { tail $OUT/tr.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/tr.json').read().strip().splitlines()[-1]); print('traced', d['ms_per_step'], d['init_ms'], d['saturate_ms'])"
python3 scripts/rpd_stats.py $OUT/tr/tr_results.db > $OUT/tr_stats.csv && head -12 $OUT/tr_stats.csv
python3 scripts/steps.py $OUT/tr/tr_results.db 5 > $OUT/tr_steps.txt && head -28 $OUT/tr_steps.txt
