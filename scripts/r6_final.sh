#!/bin/bash
# GPU session (scripts/r6_final.sh TAG): the round's record on the final source, part 1 — the whole
# -m gpu suite, a rocprofv3 kernel trace of the timed G3 bench beside an untraced run (fresh
# processes, before any PMC pass), and the PMC passes with their calibrated summary
# (profiles/pmc/r06_pmc_g3.json, which the bench line's roofline.traffic reads).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
B="bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3"
timeout -k 10 200 python $B > $OUT/u.json 2> $OUT/u.err || { tail $OUT/u.err; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o tr -- python3 $R/$B > $OUT/tr.json 2> $OUT/tr.err) || { tail $OUT/tr.err; exit 1; }
echo "untraced $(python -c "import json; d=json.load(open('$OUT/u.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])") traced $(python -c "import json; d=json.loads(open('$OUT/tr.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
python3 scripts/rpd_stats.py $OUT/tr/tr_results.db > $OUT/tr_stats.csv && head -8 $OUT/tr_stats.csv
python3 scripts/steps.py $OUT/tr/tr_results.db 5 > $OUT/tr_steps.txt
bash scripts/pmc_session.sh $1/pmc > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/$1/pmc profiles/pmc/r06_pmc_g3.json g3 > $OUT/pmc_summary.log 2>&1 || { tail $OUT/pmc_summary.log; exit 1; }
cp profiles/pmc/r06_pmc_g3.json $OUT/
grep -E "^k_expand|^k_commit |^k_jobs" $OUT/pmc_summary.log | cut -c1-400
