#!/bin/bash
# GPU session (scripts/r5_mem.sh TAG): device bytes per structure (EL_TRACE_MEM) of a whole G3
# context and of the row partitions of ×2 (aligned copies) and of one G3 on 4 ranks (strong).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
EL_TRACE_MEM=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu --no-profile --no-throughput2 > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
grep "^mem" $OUT/b.err | tail -20
EL_TRACE_MEM=1 timeout -k 10 300 python -u scripts/part_diag.py g3 1.0 2 1 weak > $OUT/w2.jsonl 2> $OUT/w2.err || { tail $OUT/w2.err; exit 1; }
grep "^mem" $OUT/w2.err | tail -20
EL_TRACE_MEM=1 timeout -k 10 300 python -u scripts/part_diag.py g3 1.0 4 1 strong > $OUT/s4.jsonl 2> $OUT/s4.err || { tail $OUT/s4.err; exit 1; }
grep "^mem" $OUT/s4.err | tail -40
