#!/bin/bash
# GPU session (scripts/r5_d.sh TAG): the copy-back tail against the process's hardware-queue count —
# engines one after another in one process (scripts/tail_diag.py) with GPU_MAX_HW_QUEUES 4 … 32.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for q in 4 8 12 16 24 32; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u scripts/tail_diag.py g3 4 whole whole rccl1 whole whole > $OUT/tail_q$q.jsonl 2> $OUT/tail_q$q.err || { tail -20 $OUT/tail_q$q.err; exit 1; }
  echo "queues $q"; cat $OUT/tail_q$q.jsonl
done
