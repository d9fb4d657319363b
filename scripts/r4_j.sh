#!/bin/bash
# GPU session (scripts/r4_j.sh TAG): parity tests, then A/B of the sorted S commit
# (EL_COMMIT_SORT=1 default vs 0) on G3 and G5 with the profiled kernel table.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
for v in 1 0; do
EL_COMMIT_SORT=$v EL_TRACE_CANDS=1 timeout -k 10 200 python -c "
from distel_amd import engine, generators
e, st = engine.classify(generators.workload('g3'))
print(st)" > $OUT/cands_$v.log 2>&1 || { tail $OUT/cands_$v.log; exit 1; }
echo "sort=$v"; grep step $OUT/cands_$v.log | head -8
done
for w in g3 g5; do
for rep in 1 2; do
  for v in 1 0; do
    EL_COMMIT_SORT=$v timeout -k 10 200 python bench.py --workload $w --no-cpu --no-throughput2 --steps 10 --warmup 3 > $OUT/ab_${w}_${v}_$rep.json 2> $OUT/ab_${w}_${v}_$rep.err || { tail $OUT/ab_${w}_${v}_$rep.err; exit 1; }
    echo "$w sort=$v $rep $(python -c "import json; d=json.load(open('$OUT/ab_${w}_${v}_$rep.json')); k=d['kernels']; print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], 'commit', k['k_commit']['ms'], 'told', k['k_commit_told']['ms'], 'expand', k['k_expand']['ms'])")"
  done
done
done
