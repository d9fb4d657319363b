#!/bin/bash
# GPU session (scripts/r5_wl_ab.sh TAG): every workload with the column order on and off
# (EL_COLUMN_ORDER=0), alternating, two rounds.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
for w in g1 g2 g5 g3x g3e; do
  for rep in 1 2; do
    for v in def id; do
      E=""; [ $v = id ] && E="EL_COLUMN_ORDER=0"
      env $E timeout -k 10 200 python bench.py --workload $w --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3 > $OUT/${w}_${v}_$rep.json 2> $OUT/${w}_${v}_$rep.err || { tail -5 $OUT/${w}_${v}_$rep.err; exit 1; }
      echo "$w $v $rep $(python -c "import json; d=json.load(open('$OUT/${w}_${v}_$rep.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['derived_axioms'])")"
    done
  done
done
