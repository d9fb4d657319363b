#!/bin/bash
# GPU session (scripts/r5_cnt.sh): G3 derived counts (against the pinned 136,499,458) with the
# column order on and off, one classification each.
for v in def id; do
  E=""; [ $v = id ] && E="EL_COLUMN_ORDER=0"
  env $E timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu --no-profile --no-throughput2 > gpurun_out/cnt_$v.json 2> gpurun_out/cnt_$v.err || { tail -5 gpurun_out/cnt_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/cnt_$v.json')); print('$v', d['derived_axioms'], d['s_facts_per_rank'], d['links_per_rank'], d['ms_per_step'])"
done
