#!/bin/bash
# GPU session (scripts/r4_p.sh TAG): what the streamed result's concurrent work (run encoding +
# DMA beside the supersteps) costs the supersteps: G3 with --copyback stream (default) vs rows
# (the copy after the fixpoint), alternating, three each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 200 python bench.py --no-cpu --no-throughput2 --no-profile --steps 10 --warmup 3 > $OUT/warm.json 2> $OUT/warm.err || { tail $OUT/warm.err; exit 1; }
for rep in 1 2 3; do
  for v in stream rows; do
    timeout -k 10 200 python bench.py --no-cpu --no-throughput2 --no-profile --steps 10 --warmup 3 --copyback $v > $OUT/b_${v}_$rep.json 2> $OUT/b_${v}_$rep.err || { tail $OUT/b_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('$OUT/b_${v}_$rep.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'])")"
  done
done
