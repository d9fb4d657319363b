#!/bin/bash
# A/B of library variants (EL_GPU_LIB) on one workload: serial latency and two-in-flight step.
set -o pipefail
TAG=${1:-libab}; W=${2:-g3}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
i=0
for lib in distel_amd/lib/libel_gpu.so "$@"; do
  for inf in 1 2; do
    i=$((i+1))
    EL_GPU_LIB=$R/$lib timeout -k 10 300 python bench.py --workload $W --inflight $inf --no-cpu --no-profile --steps 20 --warmup 5 > $OUT/r$i.json 2> $OUT/r$i.err || { tail -5 $OUT/r$i.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/r$i.json')); print('$(basename $lib) inflight $inf', d['ms_per_step'], 'ms', 'sat', d['saturate_ms'], 'lat', d['latency_ms'], round(d['value']/1e9,3), 'G/s')"
  done
done
