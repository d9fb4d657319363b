#!/bin/bash
# GPU session (scripts/r5_g.sh TAG): k_expand per rule group (EL_SPLIT_EXPAND=2: the S role once
# per rule group, then the link / activation / propagation roles) from a rocprofv3 kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
B="bench.py --no-cpu --no-profile --no-throughput2 --steps 3 --warmup 2"
(cd /tmp && EL_SPLIT_EXPAND=2 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/sp -o sp -- python3 $R/$B > $OUT/sp.json 2> $OUT/sp.err) || { tail $OUT/sp.err; exit 1; }
python3 scripts/split_expand.py "$OUT/sp/**/*.db" 2 | tee $OUT/split.txt
