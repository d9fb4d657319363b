#!/bin/bash
# GPU session (scripts/r4_r.sh TAG [VARIANTS...]): parity / export / partition / workload tests,
# then the generic G3 A/B (scripts/r4_l.sh's bench part) of NAME=ENV variants against the default.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_export.py tests/test_gpu_partition.py tests/test_gpu_workloads.py > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
shift
B="bench.py --no-cpu --no-throughput2 --steps 10 --warmup 3"
timeout -k 10 200 python $B > $OUT/warm.json 2> $OUT/warm.err || { tail $OUT/warm.err; exit 1; }
for rep in 1 2; do
  for kv in def "$@"; do
    v=${kv%%=*}; E=""; [ "$kv" != def ] && E=${kv#*=}
    env $E timeout -k 10 200 python $B > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || { tail $OUT/ab_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('$OUT/ab_${v}_$rep.json')); k=d['kernels']; print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], 'closure', k['k_closure']['ms'], 'commit', k['k_commit']['ms'], 'expand', k['k_expand']['ms'])")"
  done
done
