#!/bin/bash
# GPU session (scripts/r4_m.sh TAG): the whole -m gpu suite (slowest durations listed), then the
# bench lines of G3 / G5 / G2 at N = 1.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ --durations=12 > $OUT/t.log 2>&1
rc=$?; tail -16 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
for w in g3 g5 g2; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu --no-throughput2 --steps 10 --warmup 3 > $OUT/b_$w.json 2> $OUT/b_$w.err || { tail $OUT/b_$w.err; exit 1; }
  echo "$w $(python -c "import json; d=json.load(open('$OUT/b_$w.json')); k=d['kernels']; print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], {n: round(v['ms'],3) for n, v in k.items()})")"
done
# diagnostic: every role of k_expand / k_commit as a launch of its own (EL_SPLIT_*), traced
(cd /tmp && EL_SPLIT_EXPAND=1 EL_SPLIT_COMMIT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/sp -o sp -- python3 $R/bench.py --no-cpu --no-profile --no-throughput2 --steps 2 --warmup 1 > $OUT/sp.json 2> $OUT/sp.err) || { tail $OUT/sp.err; exit 1; }
python3 scripts/split_steps.py $OUT/sp/sp_results.db > $OUT/sp_steps.txt && head -30 $OUT/sp_steps.txt
