#!/bin/bash
# GPU session (scripts/r4_f.sh TAG): D2H copies from Python, with torch's HIP runtime or the
# system's, host or device pointer (blit = __amd_rocclr_copyBuffer in the trace); the G3 bench
# once more with the kernel trace split per rule group (EL_SPLIT_EXPAND=2).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for m in plain torch; do
  for k in hostptr devptr; do
    (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/py_${m}_$k -o p -- python3 $R/scripts/micro/d2h_py.py $m $k > $OUT/py_${m}_$k.log 2>&1) || { tail $OUT/py_${m}_$k.log; exit 1; }
    echo "$m $k: $(tail -1 $OUT/py_${m}_$k.log) | $(python3 scripts/rpd_stats.py $OUT/py_${m}_$k/p_results.db | grep -c copyBuffer) blit rows"
  done
done
(cd /tmp && EL_SPLIT_EXPAND=2 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/split -o s -- python3 $R/bench.py --no-cpu --no-profile --no-throughput2 --steps 3 --warmup 1 > $OUT/split.json 2> $OUT/split.err) || { tail $OUT/split.err; exit 1; }
python3 scripts/split_expand.py "$OUT/split/s_results.db" 2
