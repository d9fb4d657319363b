#!/bin/bash
# GPU session (scripts/r4_k.sh TAG): parity / export / partition tests; G3 A/B: init facts on the
# side stream (default) vs inline, lane merges off, stream priorities, summary-clear grids; a kernel
# trace of the G3 bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_export.py tests/test_gpu_partition.py > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
B="bench.py --no-cpu --no-throughput2 --steps 10 --warmup 3"
for rep in 1 2; do
  for v in def inline nolanes prio grid256 grid512; do
    E=""; [ $v = inline ] && E="EL_INIT_INLINE=1"; [ $v = prio ] && E="EL_STREAM_PRIO=1"; [ $v = nolanes ] && E="EL_CLOSURE_LANES=0"
    [ $v = grid256 ] && E="EL_CLEAR_GRID=256"; [ $v = grid512 ] && E="EL_CLEAR_GRID=512"
    env $E timeout -k 10 200 python $B > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || { tail $OUT/ab_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('$OUT/ab_${v}_$rep.json')); k=d['kernels']; print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], 'closure', k['k_closure']['ms'], 'commit', k['k_commit']['ms'])")"
  done
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o tr -- python3 $R/bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3 > $OUT/tr.json 2> $OUT/tr.err) || { tail $OUT/tr.err; exit 1; }
echo "trace $(python -c "import json; d=json.loads(open('$OUT/tr.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
python3 scripts/rpd_stats.py $OUT/tr/tr_results.db | head -14
python3 scripts/steps.py $OUT/tr/tr_results.db 5 | head -8
