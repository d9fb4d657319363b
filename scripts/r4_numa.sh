#!/bin/bash
# GPU session (scripts/r4_numa.sh TAG): the box's NUMA layout, then G3 bench runs in fresh
# processes alternating EL_NUMA_BIND=1 (default) and 0, four each: does the copy-back tail
# (copyback_ms, the streamed result's D2H) depend on where the page-locked buffers live?
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
cat /sys/devices/system/node/online > $OUT/numa.txt 2>&1
for n in /sys/devices/system/node/node*; do echo "$n $(cat $n/cpulist)" >> $OUT/numa.txt; done
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))" >> $OUT/numa.txt
cat $OUT/numa.txt
for rep in 1 2 3 4; do
  for v in 1 0; do
    EL_NUMA_BIND=$v timeout -k 10 200 python bench.py --no-cpu --no-throughput2 --no-profile --steps 10 --warmup 3 > $OUT/b_${v}_$rep.json 2> $OUT/b_${v}_$rep.err || { tail $OUT/b_${v}_$rep.err; exit 1; }
    echo "bind=$v $rep $(python -c "import json; d=json.load(open('$OUT/b_${v}_$rep.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], d.get('numa'))")"
  done
done
