#!/bin/bash
# Per-step candidate counts (EL_TRACE_CANDS) and a rocprofv3 kernel timeline of one workload.
# Usage: scripts/r2_trace.sh TAG WORKLOAD
set -o pipefail
TAG=${1:-trace}; W=${2:-g3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
EL_TRACE_CANDS=1 timeout -k 10 300 python bench.py --workload $W --no-cpu --no-profile --steps 1 --warmup 0 > $OUT/cands.json 2> $OUT/cands.err || { tail -5 $OUT/cands.err; exit 1; }
grep -c step $OUT/cands.err
bash scripts/r2_prof.sh $TAG $W > /dev/null
