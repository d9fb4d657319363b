#!/bin/bash
# Per-step candidate counts (EL_TRACE_CANDS) of G3 and G2, serial schedule, plus the default bench line.
set -o pipefail
TAG=${1:-trace}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for w in g3 g2; do
  EL_TRACE_CANDS=1 timeout -k 10 300 python bench.py --workload $w --inflight 1 --no-cpu --no-profile --steps 1 --warmup 0 > $OUT/c_$w.json 2> $OUT/c_$w.err || { tail -5 $OUT/c_$w.err; exit 1; }
done
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 > $OUT/g3.json 2> $OUT/g3.err || { tail -5 $OUT/g3.err; exit 1; }
cat $OUT/g3.json
