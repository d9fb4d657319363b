#!/bin/bash
# GPU session (scripts/r5_q.sh TAG): incremental + told-cycle tests, the increment's phases,
# and G3E (told cycles) timed beside G3 with a kernel trace of G3E.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_incremental.py "tests/test_gpu_workloads.py::test_g3e_told_cycles" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
EL_TRACE_INC=1 timeout -k 10 300 python bench.py --increment 0.01 --steps 3 --warmup 1 --no-cpu --no-profile --no-throughput2 > $OUT/b1.json 2> $OUT/b1.err || { tail -20 $OUT/b1.err; exit 1; }
grep migrate $OUT/b1.err | tail -7
python -c "import json; d=json.load(open('$OUT/b1.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms']); i=d['increment']; print({k: i[k] for k in ('index_ms','upload_ms','migrate_ms','saturate_ms','classification_ms','retrigger','vs_full_classification')})"
for w in g3e g3; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu --no-profile --no-throughput2 > $OUT/b_$w.json 2> $OUT/b_$w.err || { tail -20 $OUT/b_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$w.json')); print('$w', d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], d['supersteps'], d['derived_axioms'])"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tre -o tre -- python3 $R/bench.py --workload g3e --steps 3 --warmup 1 --no-cpu --no-profile --no-throughput2 > $OUT/tre.json 2> $OUT/tre.err) || { tail $OUT/tre.err; exit 1; }
python3 scripts/rpd_stats.py $OUT/tre/tre_results.db > $OUT/tre_stats.csv && head -14 $OUT/tre_stats.csv
