#!/bin/bash
# GPU session (scripts/r3_c.sh TAG): D2H alignment micro (+ kernel trace), the partition test
# files, and a 2-rank rehearsal of the bench's exchange leg on one GPU (host transport).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 60 ./scripts/micro/d2h_align > $OUT/align.txt 2>&1 || { cat $OUT/align.txt; exit 1; }
cat $OUT/align.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 90 rocprofv3 --kernel-trace -d $OUT/alignprof -o a -- $R/scripts/micro/d2h_align > $OUT/alignprof.log 2>&1) || { tail $OUT/alignprof.log; exit 1; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_xproc.py tests/test_gpu_partition.py > $OUT/part.log 2>&1
rc=$?; tail -4 $OUT/part.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/part.log | head -20; exit $rc; }
EL_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --transport host --steps 3 --warmup 1 --no-cpu --no-profile > $OUT/b2.json 2> $OUT/b2.err || { tail -20 $OUT/b2.err; exit 1; }
cat $OUT/b2.json
