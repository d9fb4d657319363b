#!/bin/bash
# Launch-shape sweep on G2/G3: scripts/sweep.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
for cfg in "1024 1024 512" "512 512 512" "256 256 256" "512 256 256" "256 512 256"; do
  set -- $cfg
  for w in g2 g3; do
    EL_COMMIT_BLOCKS=$1 EL_JOBS_BLOCKS=$2 EL_SCATTER_BLOCKS=$3 timeout -k 10 300 python bench.py --workload $w --no-cpu --no-profile --steps 5 --warmup 2 > $OUT/b_${1}_${2}_${3}_$w.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$OUT/b_${1}_${2}_${3}_$w.json')); print('$cfg $w', d['ms_per_step'])"
  done
done
