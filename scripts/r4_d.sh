#!/bin/bash
# GPU session (scripts/r4_d.sh TAG): which D2H copies run as blit kernels (micro, one trace per
# case); G3 bench A/B (default, host-pointer D2H copies, no block summary, 128-record wave queues);
# rocprofv3 kernel traces of the timed G3 bench (default and host-pointer copies).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for c in A B C D E; do
  (cd /tmp && timeout -k 10 60 rocprofv3 --kernel-trace --stats -d $OUT/mode_$c -o m -- $R/scripts/micro/d2h_mode $c > $OUT/mode_$c.log 2>&1) || { tail $OUT/mode_$c.log; exit 1; }
  echo "case $c: $(grep -E '^[A-E] ' $OUT/mode_$c.log) | blits: $(find $OUT/mode_$c -name '*kernel_stats.csv' | xargs grep -h copyBuffer | cut -d, -f1-3)"
done
B="python bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3"
for rep in 1 2; do
  for v in def hostptr nosumm wq128; do
    case $v in
      def) E="";; hostptr) E="EL_DMA_HOSTPTR=1";; nosumm) E="EL_NO_SUMMARY=1";; wq128) E="EL_GPU_LIB=$R/distel_amd/lib/libel_gpu_wq128.so";;
    esac
    env $E timeout -k 10 200 $B > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || { tail $OUT/ab_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('$OUT/ab_${v}_$rep.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
  done
done
for v in def hostptr; do
  E=""; [ $v = hostptr ] && E="EL_DMA_HOSTPTR=1"
  (cd /tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_$v -o tr -- python3 $R/bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3 > $OUT/tr_$v.json 2> $OUT/tr_$v.err) || { tail $OUT/tr_$v.err; exit 1; }
  echo "trace $v $(python -c "import json; d=json.loads(open('$OUT/tr_$v.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
  head -12 $(find $OUT/tr_$v -name '*kernel_stats.csv' | head -1) | cut -d, -f1-5
done
