#!/bin/bash
# GPU session (scripts/r4_g2trace.sh TAG): rocprofv3 kernel trace of the timed G2 bench beside an
# untraced run, and the per-superstep split of one classification (scripts/steps.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
B="bench.py --workload g2 --no-cpu --no-profile --no-throughput2 --steps 20 --warmup 3"
timeout -k 10 200 python $B > $OUT/u.json 2> $OUT/u.err || { tail $OUT/u.err; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o tr -- python3 $R/$B > $OUT/tr.json 2> $OUT/tr.err) || { tail $OUT/tr.err; exit 1; }
echo "untraced $(python -c "import json; d=json.load(open('$OUT/u.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])") traced $(python -c "import json; d=json.loads(open('$OUT/tr.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
python3 scripts/rpd_stats.py $OUT/tr/tr_results.db > $OUT/tr_stats.csv && head -12 $OUT/tr_stats.csv
python3 scripts/steps.py $OUT/tr/tr_results.db 10 > $OUT/tr_steps.txt
cp $OUT/tr/tr_results.db $OUT/g2.db
