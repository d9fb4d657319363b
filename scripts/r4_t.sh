#!/bin/bash
# GPU session (scripts/r4_t.sh TAG VARIANT [AB_VARIANTS...]): the parity / export / workload tests on
# library variant VARIANT (EL_LIB_VARIANT, scripts/build_variant.sh), then the G3 A/B of the default
# library against every listed variant, alternating, three rounds.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
EL_LIB_VARIANT=$2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_export.py tests/test_gpu_workloads.py > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
shift 2
B="bench.py --no-cpu --no-throughput2 --steps 10 --warmup 3"
timeout -k 10 200 python $B > $OUT/warm.json 2> $OUT/warm.err || { tail $OUT/warm.err; exit 1; }
for rep in 1 2 3; do
  for v in def "$@"; do
    E=""; [ "$v" != def ] && E="EL_LIB_VARIANT=$v"
    env $E timeout -k 10 200 python $B > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || { tail $OUT/ab_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('$OUT/ab_${v}_$rep.json')); k=d['kernels']; print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], 'closure', k['k_closure']['ms'], 'commit', k['k_commit']['ms'], 'expand', k['k_expand']['ms'])")"
  done
done
