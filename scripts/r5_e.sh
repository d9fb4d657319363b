#!/bin/bash
# GPU session (scripts/r5_e.sh TAG): the copy-back tail with and without NUMA binding (12 queues).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for n in 1 0 1; do
  NUMA=$n GPU_MAX_HW_QUEUES=12 timeout -k 10 300 python -u scripts/tail_diag.py g3 4 whole whole rccl1 > $OUT/tail_n$n.jsonl 2> $OUT/tail_n$n.err || { tail -20 $OUT/tail_n$n.err; exit 1; }
  echo "numa $n"; cat $OUT/tail_n$n.jsonl
done
