#!/bin/bash
# Extra workloads (informational): G3 and G5 single-GPU classification.
set -o pipefail
TAG=${1:-extra}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for w in g5 g3 g1; do
  timeout -k 10 400 python bench.py --workload $w --steps 3 --warmup 1 --verbose > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  rc=$?; echo "bench $w rc=$rc"; head -c 1500 $OUT/bench_$w.json; echo
  [ $rc -eq 0 ] || exit $rc
done
