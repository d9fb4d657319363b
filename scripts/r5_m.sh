#!/bin/bash
# GPU session (scripts/r5_m.sh TAG): the plain G3 bench with the D2H probe before the engine
# (EL_D2H_PROBE=both) against after it (end, the default), alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for i in 1 2 3; do
  for p in end both; do
    EL_D2H_PROBE=$p timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-profile --no-throughput2 > $OUT/b_${p}_$i.json 2> $OUT/b_${p}_$i.err || { tail -20 $OUT/b_${p}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${p}_$i.json')); print('$p', d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], d.get('d2h_gbs'))"
  done
done
