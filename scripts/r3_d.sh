#!/bin/bash
# GPU session (scripts/r3_d.sh TAG): which HIP runtime makes D2H a blit kernel (the D2H micro on
# the system runtime vs torch's bundled one, with runtime knobs), the partition test files, and a
# 2-rank rehearsal of the bench's exchange leg on one GPU (host transport).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
TL=$(python -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
export TMPDIR=/tmp
for v in sys torch torch_bet1 torch_bet2 torch_sdma1; do
  case $v in
    sys) E="";;
    torch) E="LD_LIBRARY_PATH=$TL";;
    torch_bet1) E="LD_LIBRARY_PATH=$TL GPU_BLIT_ENGINE_TYPE=1";;
    torch_bet2) E="LD_LIBRARY_PATH=$TL GPU_BLIT_ENGINE_TYPE=2";;
    torch_sdma1) E="LD_LIBRARY_PATH=$TL HSA_ENABLE_SDMA=1";;
  esac
  (cd /tmp && env $E timeout -k 10 90 rocprofv3 --kernel-trace -d $OUT/p_$v -o a -- $R/scripts/micro/d2h_align > $OUT/p_$v.log 2>&1) || { tail $OUT/p_$v.log; exit 1; }
  echo "== $v"; grep -E "aligned|off4 both" $OUT/p_$v.log | head -2
  python3 scripts/rpd_stats.py "$OUT/p_$v/**/*.db" | head -4
done
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_xproc.py tests/test_gpu_partition.py > $OUT/part.log 2>&1
rc=$?; tail -4 $OUT/part.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/part.log | head -20; exit $rc; }
EL_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --transport host --steps 3 --warmup 1 --no-cpu --no-profile > $OUT/b2.json 2> $OUT/b2.err || { tail -20 $OUT/b2.err; exit 1; }
cat $OUT/b2.json
