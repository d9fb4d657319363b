#!/bin/bash
# A/B of configurations "LIB [ENV=V ...]" (LIB relative to the repo) on one workload: serial and two in flight.
# Usage: scripts/r2_cfg_ab.sh TAG WORKLOAD "cfg1" "cfg2" ...
set -o pipefail
TAG=${1:-cfgab}; W=${2:-g3}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
i=0
for cfg in "$@"; do
  set -- $cfg
  lib=$1; shift
  for inf in 1 2; do
    i=$((i+1))
    env EL_GPU_LIB=$R/$lib "$@" timeout -k 10 300 python bench.py --workload $W --inflight $inf --no-cpu --no-profile --steps 20 --warmup 5 > $OUT/r$i.json 2> $OUT/r$i.err || { tail -5 $OUT/r$i.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/r$i.json')); print('$cfg', 'inflight $inf', d['ms_per_step'], 'ms', 'sat', d['saturate_ms'], 'lat', d['latency_ms'], round(d['value']/1e9,3), 'G/s')"
  done
done
