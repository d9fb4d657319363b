#!/bin/bash
# GPU session (scripts/r6_small_ab.sh TAG VARIANT...): the small workloads (G1, G2, G5; WS env
# overrides) with the default build against variants (NAME=ENV or lib:TAG), alternating, three
# rounds: ms_per_step, init and saturate.  CB: --copyback (default auto; stream for a variant
# built from a source without the packed stream).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
shift
for w in ${WS:-g1 g2 g5}; do
  B="bench.py --no-cpu --no-profile --no-throughput2 --steps 20 --warmup 5 --workload $w --copyback ${CB:-auto}"
  timeout -k 10 200 python $B > $OUT/warm_$w.json 2> $OUT/warm_$w.err || { tail $OUT/warm_$w.err; exit 1; }
  for rep in 1 2 3; do
    for kv in def "$@"; do
      v=${kv%%=*}; E=""
      case "$kv" in def) ;; lib:*) v=${kv#lib:}; E="EL_LIB_VARIANT=$v" ;; *) E=${kv#*=} ;; esac
      env $E timeout -k 10 200 python $B > $OUT/${w}_${v}_$rep.json 2> $OUT/${w}_${v}_$rep.err || { tail $OUT/${w}_${v}_$rep.err; exit 1; }
      echo "$w $v $rep $(python -c "import json; d=json.load(open('$OUT/${w}_${v}_$rep.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_encoding'])")"
    done
  done
done
