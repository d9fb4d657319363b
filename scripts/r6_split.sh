#!/bin/bash
# GPU session (scripts/r6_split.sh TAG [workload]): k_expand time per rule group and superstep
# (EL_SPLIT_EXPAND=2, rocprofv3 kernel trace of the bench).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
W=${2:-g3}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
export EL_SPLIT_EXPAND=2
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o tr -- python3 $R/bench.py --workload $W --steps 2 --warmup 1 --no-cpu --no-profile --no-throughput2 > $OUT/b.json 2> $OUT/b.err) || { tail $OUT/b.err; exit 1; }
python3 scripts/split_rules_steps.py $OUT/tr/tr_results.db > $OUT/split.txt && cat $OUT/split.txt
