#!/bin/bash
# GPU session (scripts/r5_r.sh TAG): the whole GPU suite, then G3E (told cycles) and G3 timed.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for w in g3e g3; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu --no-profile --no-throughput2 > $OUT/b_$w.json 2> $OUT/b_$w.err || { tail -20 $OUT/b_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$w.json')); print('$w', d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], d['supersteps'], d['derived_axioms'])"
done
