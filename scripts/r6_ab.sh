#!/bin/bash
# GPU session (scripts/r6_ab.sh TAG "pytest -k expr" VARIANT...): parity subset first (skipped when
# the expression is "-"), then the G3 A/B of the default build against variants (scripts/r4_ab.sh
# conventions: NAME=ENV or lib:TAG), alternating, three rounds, then the per-rule k_expand split
# of the default build.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
K=$2
shift 2
if [ "$K" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $OUT/t.log 2>&1
  rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
fi
B="bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3 --workload ${W:-g3}"
timeout -k 10 200 python $B > $OUT/warm.json 2> $OUT/warm.err || { tail $OUT/warm.err; exit 1; }
for rep in 1 2 3; do
  for kv in def "$@"; do
    v=${kv%%=*}; E=""
    case "$kv" in def) ;; lib:*) v=${kv#lib:}; E="EL_LIB_VARIANT=$v" ;; *) E=${kv#*=} ;; esac
    env $E timeout -k 10 200 python $B > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || { tail $OUT/ab_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('$OUT/ab_${v}_$rep.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
  done
done
export EL_SPLIT_EXPAND=2
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/sp -o tr -- python3 $R/bench.py --workload ${W:-g3} --steps 2 --warmup 1 --no-cpu --no-profile --no-throughput2 > $OUT/sp.json 2> $OUT/sp.err) || { tail $OUT/sp.err; exit 1; }
python3 scripts/split_rules_steps.py $OUT/sp/tr_results.db > $OUT/split.txt && head -8 $OUT/split.txt && tail -1 $OUT/split.txt
