#!/bin/bash
# GPU session (scripts/r5_inct.sh TAG): kernel trace of the increment leg (one base
# classification, then el_add_axioms + el_saturate of a 1 % G3 increment) and its table.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
B="bench.py --increment 0.01 --steps 1 --warmup 0 --no-cpu --no-profile --no-throughput2"
(cd /tmp && EL_TRACE_INC=1 EL_TRACE_GROW=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o tr -- python3 $R/$B > $OUT/tr.json 2> $OUT/tr.err) || { tail $OUT/tr.err; exit 1; }
grep "migrate\|grow\|increment sat" $OUT/tr.err | tail -30
python3 scripts/inc_trace.py "$OUT/tr/**/tr_results.db" > $OUT/inc_trace.txt && head -30 $OUT/inc_trace.txt
