#!/bin/bash
# GPU session (scripts/r5_split.sh TAG): per-role k_expand / k_commit times per superstep
# (EL_SPLIT_EXPAND / EL_SPLIT_COMMIT, rocprofv3 kernel trace) with the column order on and off.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for v in def id; do
  E="EL_SPLIT_EXPAND=1 EL_SPLIT_COMMIT=1"; [ $v = id ] && E="$E EL_COLUMN_ORDER=0"
  (cd /tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/$v -o tr -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-profile --no-throughput2 > $OUT/$v.json 2> $OUT/$v.err) || { tail $OUT/$v.err; exit 1; }
  python3 scripts/split_steps.py $OUT/$v/tr_results.db > $OUT/${v}_split.txt && echo "== $v" && head -12 $OUT/${v}_split.txt
done
