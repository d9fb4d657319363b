#!/bin/bash
# GPU session (scripts/r5_inc3.sh TAG): the increment leg with several repetitions and the
# per-phase traces (EL_TRACE_INC, EL_TRACE_GROW), untraced by rocprof.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
EL_TRACE_INC=1 EL_TRACE_GROW=1 timeout -k 10 300 python bench.py --increment 0.01 --steps 5 --warmup 1 --no-cpu --no-profile --no-throughput2 > $OUT/inc.json 2> $OUT/inc.err || { tail -20 $OUT/inc.err; exit 1; }
grep "migrate\|grow\|re-trigger\|increment sat" $OUT/inc.err | tail -80
