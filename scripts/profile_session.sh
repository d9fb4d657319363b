#!/bin/bash
# Profile session for one source version (no parity suite: run quick_gpu.sh for that first).
#   G2 bench line with the CPU leg, rocprofv3 kernel stats + kernel trace of the same command,
#   FETCH_SIZE / WRITE_SIZE passes (one counter group per pass) for G2 and G3, G3/G5/G1 lines.
# Usage: scripts/profile_session.sh TAG.  Every GPU step has its own limit; the chain stops at
# the first failure.
set -o pipefail
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python bench.py --verbose > $OUT/bench_g2.json 2> $OUT/bench_g2.err
rc=$?; echo "bench g2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench_g2.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --no-cpu > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/prof.log; exit $rc; }
for w in g2 g3; do
  i=0; mkdir -p $OUT/pmc_$w
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$w/p$i -o run -- python3 $R/bench.py --workload $w --no-cpu --no-profile --steps 1 --warmup 0 > $OUT/pmc_$w/p$i.log 2>&1
    rc=$?; echo "pmc $w $grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
cd $R
for w in g3 g5 g1; do
  timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu > $OUT/bench_$w.json 2> $OUT/bench_$w.err
  rc=$?; echo "bench $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
