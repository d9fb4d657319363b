#!/bin/bash
# GPU session (scripts/r5_n.sh TAG): the plain G3 bench, this source against the round-4 library
# (EL_LIB_VARIANT=r4), alternating; D2H probed at the end of each run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in def r4; do
    E=""; [ $v = r4 ] && E="EL_LIB_VARIANT=r4"
    env $E timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-profile --no-throughput2 > $OUT/b_${v}_$i.json 2> $OUT/b_${v}_$i.err || { tail -20 $OUT/b_${v}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${v}_$i.json')); print('$v', d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], d.get('d2h_gbs'), d.get('lib'))"
  done
done
