#!/bin/bash
# GPU session (scripts/r5_final.sh TAG): the round's record on the final source — the whole -m gpu
# suite, a rocprofv3 kernel trace of the timed G3 bench beside an untraced run (fresh processes,
# before any PMC pass), the PMC passes with their calibrated summary (profiles/pmc/r05_pmc_g3.json,
# which the bench line's roofline.traffic reads), the default bench line (G3, N = 1, cpu_baseline
# with the whole-G3 one-core run) and the bench lines of the other workloads (G3E too), and the 1 % G3 increment line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
B="bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3"
timeout -k 10 200 python $B > $OUT/u.json 2> $OUT/u.err || { tail $OUT/u.err; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o tr -- python3 $R/$B > $OUT/tr.json 2> $OUT/tr.err) || { tail $OUT/tr.err; exit 1; }
echo "untraced $(python -c "import json; d=json.load(open('$OUT/u.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])") traced $(python -c "import json; d=json.loads(open('$OUT/tr.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
python3 scripts/rpd_stats.py $OUT/tr/tr_results.db > $OUT/tr_stats.csv && head -8 $OUT/tr_stats.csv
python3 scripts/steps.py $OUT/tr/tr_results.db 5 > $OUT/tr_steps.txt
bash scripts/pmc_session.sh $1/pmc > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/$1/pmc profiles/pmc/r05_pmc_g3.json g3 > $OUT/pmc_summary.log 2>&1 || { tail $OUT/pmc_summary.log; exit 1; }
cp profiles/pmc/r05_pmc_g3.json $OUT/
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
for w in g1 g2 g5 g3x g3e; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu --steps 10 --warmup 3 > $OUT/b_$w.json 2> $OUT/b_$w.err || { tail $OUT/b_$w.err; exit 1; }
  echo "$w $(python -c "import json; d=json.load(open('$OUT/b_$w.json')); print(d['ms_per_step'], d['value'], d['init_ms'], d['saturate_ms'])")"
done
timeout -k 10 300 python bench.py --increment 0.01 --steps 5 --warmup 1 --no-cpu --no-profile --no-throughput2 > $OUT/inc.json 2> $OUT/inc.err || { tail $OUT/inc.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/inc.json')); i=d['increment']; print('increment', {k: i[k] for k in ('index_ms','upload_ms','migrate_ms','saturate_ms','classification_ms','retrigger','vs_full_classification')})"
