#!/bin/bash
# GPU session (scripts/r5_inc4.sh TAG): kernel trace of the increment leg over several
# repetitions (scripts/inc_steps.py: each re-trigger step's kernels).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
(cd /tmp && EL_TRACE_INC=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o tr -- python3 $R/bench.py --increment 0.01 --steps 4 --warmup 0 --no-cpu --no-profile --no-throughput2 > $OUT/inc.json 2> $OUT/inc.err) || { tail -20 $OUT/inc.err; exit 1; }
grep "increment sat" $OUT/inc.err
python3 scripts/inc_steps.py "$OUT/tr/tr_results.db" > $OUT/steps.txt && cat $OUT/steps.txt
