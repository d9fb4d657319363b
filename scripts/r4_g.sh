#!/bin/bash
# GPU session (scripts/r4_g.sh TAG): G3 bench A/B torch's HIP runtime vs the system one
# (EL_HIP_RUNTIME=system: SDMA copies instead of blit kernels), and the kernel trace of each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
B="bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3"
for rep in 1 2; do
  for v in torch system; do
    EL_HIP_RUNTIME=$v timeout -k 10 200 python $B > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || { tail $OUT/ab_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('$OUT/ab_${v}_$rep.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
  done
done
for v in system torch; do
  (cd /tmp && EL_HIP_RUNTIME=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_$v -o tr -- python3 $R/$B > $OUT/tr_$v.json 2> $OUT/tr_$v.err) || { tail $OUT/tr_$v.err; exit 1; }
  echo "trace $v $(python -c "import json; d=json.loads(open('$OUT/tr_$v.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
  python3 scripts/rpd_stats.py $OUT/tr_$v/tr_results.db | head -8
done
EL_HIP_RUNTIME=system timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-throughput2 > $OUT/full_system.json 2> $OUT/full_system.err || { tail $OUT/full_system.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/full_system.json')); print(d['ms_per_step'], d['roofline'], d['cpu_baseline'])"
