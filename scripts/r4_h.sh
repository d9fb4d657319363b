#!/bin/bash
# GPU session (scripts/r4_h.sh TAG): parity / export / partition tests on the current source; G3
# A/B of deferred small stream flushes; per-step candidate counts; a kernel trace of the G3 bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_export.py tests/test_gpu_partition.py > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
B="bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3"
for rep in 1 2; do
  for v in def every; do
    E=""; [ $v = every ] && E="EL_STREAM_MIN=1"
    env $E timeout -k 10 200 python $B > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || { tail $OUT/ab_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('$OUT/ab_${v}_$rep.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'])")"
  done
done
EL_TRACE_CANDS=1 timeout -k 10 200 python -c "
from distel_amd import engine, generators
e, st = engine.classify(generators.workload('g3'))
print(st)" > $OUT/cands.log 2>&1 || { tail $OUT/cands.log; exit 1; }
grep step $OUT/cands.log | head -24
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o tr -- python3 $R/$B > $OUT/tr.json 2> $OUT/tr.err) || { tail $OUT/tr.err; exit 1; }
echo "trace $(python -c "import json; d=json.loads(open('$OUT/tr.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
python3 scripts/rpd_stats.py $OUT/tr/tr_results.db | head -12
timeout -k 10 120 scripts/micro/commit_rate > $OUT/commit_rate.txt 2>&1 || { tail $OUT/commit_rate.txt; exit 1; }
cat $OUT/commit_rate.txt
