#!/bin/bash
# GPU session (scripts/r4_e.sh TAG): does the hardware-queue count decide blit vs SDMA for the
# streamed copies?  The D2H micro with 12 queues; the G3 bench (untraced and traced) with 4.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for q in 4 12; do
  (cd /tmp && GPU_MAX_HW_QUEUES=$q timeout -k 10 60 rocprofv3 --kernel-trace --stats -d $OUT/mode_q$q -o m -- $R/scripts/micro/d2h_mode A > $OUT/mode_q$q.log 2>&1) || { tail $OUT/mode_q$q.log; exit 1; }
  echo "micro A queues $q: $(grep -E '^A ' $OUT/mode_q$q.log)"; python3 scripts/rpd_stats.py $OUT/mode_q$q/m_results.db | head -4
done
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3 > $OUT/b_q$q.json 2> $OUT/b_q$q.err || { tail $OUT/b_q$q.err; exit 1; }
  echo "bench queues $q $(python -c "import json; d=json.load(open('$OUT/b_q$q.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
  (cd /tmp && GPU_MAX_HW_QUEUES=$q timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_q$q -o tr -- python3 $R/bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3 > $OUT/tr_q$q.json 2> $OUT/tr_q$q.err) || { tail $OUT/tr_q$q.err; exit 1; }
  echo "trace queues $q $(python -c "import json; d=json.loads(open('$OUT/tr_q$q.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
  python3 scripts/rpd_stats.py $OUT/tr_q$q/tr_results.db | head -6
done
