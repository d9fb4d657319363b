#!/bin/bash
# GPU session (scripts/r3_b.sh TAG): D2H engine micro (+ its kernel trace), the cross-process
# partition tests, and a 2-rank rehearsal of the bench's exchange leg on one GPU (host transport).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
env | grep -iE "sdma|^hip|^hsa|^gpu_|^roc|blit" > $OUT/env.txt
timeout -k 10 120 ./scripts/micro/d2h_engine > $OUT/d2h.txt 2>&1 || { cat $OUT/d2h.txt; exit 1; }
cat $OUT/d2h.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/d2hprof -o d2h -- $R/scripts/micro/d2h_engine > $OUT/d2hprof.log 2>&1) || { tail $OUT/d2hprof.log; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_xproc.py > $OUT/xproc.log 2>&1
rc=$?; tail -8 $OUT/xproc.log; [ $rc -eq 0 ] || exit $rc
EL_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --transport host --steps 3 --warmup 1 --no-cpu --no-profile > $OUT/b2.json 2> $OUT/b2.err || { tail -20 $OUT/b2.err; exit 1; }
cat $OUT/b2.json
