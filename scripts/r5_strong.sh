#!/bin/bash
# GPU session (scripts/r5_strong.sh TAG): strong-scaling diagnostics — ONE G3 ontology on 2 and 4
# unaligned row partitions (LOCAL transport, one process), per-rank kernel tables and the union's
# closure digest against the pinned one.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for k in ${PARTS:-2 4}; do
  timeout -k 10 400 python -u scripts/part_diag.py ${WL:-g3} ${SCALE:-1.0} $k ${STEPS:-2} strong > $OUT/strong$k.jsonl 2> $OUT/strong$k.err || { tail -20 $OUT/strong$k.err; exit 1; }
done
tail -c 3000 $OUT/strong*.jsonl | cut -c1-600
