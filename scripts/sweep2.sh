#!/bin/bash
# Launch-shape sweep (scripts/sweep2.sh TAG): EL_EXPAND_BLOCKS / EL_COMMIT_BLOCKS / EL_JOBS_BLOCKS on G2/G3/G5
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
for cfg in "1024 1024 1024" "1024 1024 256" "1024 1024 512" "2048 1024 1024" "1024 2048 1024" "512 1024 512"; do
  set -- $cfg
  for w in g2 g5 g3; do
    EL_EXPAND_BLOCKS=$1 EL_COMMIT_BLOCKS=$2 EL_JOBS_BLOCKS=$3 timeout -k 10 200 python bench.py --workload $w --no-cpu --no-profile --steps 5 --warmup 2 > $OUT/b_${1}_${2}_${3}_$w.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$OUT/b_${1}_${2}_${3}_$w.json')); print('$cfg $w', d['ms_per_step'])"
  done
done
