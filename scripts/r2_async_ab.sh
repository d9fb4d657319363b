#!/bin/bash
# A/B of the copy-back's footprint under the other engine's saturation (2 engines in flight).
set -o pipefail
TAG=${1:-asyncab}; W=${2:-g3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
i=0
for env in "X=0" "EL_READOUT_MIN=0"; do
  i=$((i+1))
  env $env timeout -k 10 300 python bench.py --workload $W --inflight 2 --no-cpu --no-profile --steps 20 --warmup 5 > $OUT/r$i.json 2> $OUT/r$i.err || { tail -5 $OUT/r$i.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/r$i.json')); print('$env', d['ms_per_step'], 'ms', 'sat', d['saturate_ms'], 'lat', d['latency_ms'], 'copy', d['copyback_ms'], round(d['value']/1e9,3), 'G/s')"
done
