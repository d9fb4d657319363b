#!/bin/bash
# GPU session (scripts/r5_mem4.sh TAG): device bytes per structure (EL_TRACE_MEM) of the
# configs[3] shape at full size on fewer copies — ×4 of G3 on 4 aligned partitions in one process
# (×8 at full size does not fit one GPU) — for the per-GPU projection at ×8.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
EL_TRACE_MEM=1 timeout -k 10 500 python -u scripts/part_diag.py g3 1.0 4 1 weak > $OUT/weak4.jsonl 2> $OUT/weak4.err || { tail -20 $OUT/weak4.err; exit 1; }
grep "^mem rank" $OUT/weak4.err | sort -u
grep -A20 "^mem rank 3 rows" $OUT/weak4.err | tail -21
EL_TRACE_MEM=1 timeout -k 10 500 python -u scripts/part_diag.py g3 0.5 8 1 weak > $OUT/weak8_half.jsonl 2> $OUT/weak8_half.err || { tail -20 $OUT/weak8_half.err; exit 1; }
grep "^mem rank" $OUT/weak8_half.err | sort -u | tail -3
grep -A20 "^mem rank 7 rows" $OUT/weak8_half.err | tail -21
