#!/bin/bash
# Repeated bench lines (scripts/rep_bench.sh TAG WORKLOAD REPS): run-to-run spread of ms_per_step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
for i in $(seq ${3:-3}); do
  timeout -k 10 200 env $4 python bench.py --workload $2 --no-cpu --no-profile --steps 10 --warmup 3 > $OUT/b.json 2>> $OUT/err.log || exit 1
  echo "$2 $4 $(python -c "import json; d=json.load(open('$OUT/b.json')); print(d['ms_per_step'])")"
done
