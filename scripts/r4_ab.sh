#!/bin/bash
# GPU session (scripts/r4_ab.sh TAG VARIANT...): G3 A/B of the default build against variants,
# alternating, three rounds.  A variant is NAME=ENV (an environment setting) or lib:TAG (the
# library variant EL_LIB_VARIANT=TAG, scripts/build_variant.sh); then one rocprofv3 kernel trace
# of the default build (--stats) for the per-kernel times of the background streams.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
shift
B="bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3"
timeout -k 10 200 python $B > $OUT/warm.json 2> $OUT/warm.err || { tail $OUT/warm.err; exit 1; }
for rep in 1 2 3; do
  for kv in def "$@"; do
    v=${kv%%=*}; E=""
    case "$kv" in def) ;; lib:*) v=${kv#lib:}; E="EL_LIB_VARIANT=$v" ;; *) E=${kv#*=} ;; esac
    env $E timeout -k 10 200 python $B > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || { tail $OUT/ab_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('$OUT/ab_${v}_$rep.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
  done
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o tr -- python3 $R/$B > $OUT/tr.json 2> $OUT/tr.err) || { tail $OUT/tr.err; exit 1; }
python3 scripts/rpd_stats.py $OUT/tr/tr_results.db > $OUT/tr_stats.csv && grep -E "k_clear_summ|k_level|k_expand" $OUT/tr_stats.csv
