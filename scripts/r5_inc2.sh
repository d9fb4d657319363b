#!/bin/bash
# GPU session (scripts/r5_inc2.sh TAG): the increment's phases (EL_TRACE_INC) and the plain bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
EL_TRACE_INC=1 timeout -k 10 300 python bench.py --increment 0.01 --steps 3 --warmup 1 --no-cpu --no-profile --no-throughput2 > $OUT/b1.json 2> $OUT/b1.err || { tail -20 $OUT/b1.err; exit 1; }
grep migrate $OUT/b1.err | tail -8
python -c "import json; d=json.load(open('$OUT/b1.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], d.get('d2h_gbs')); i=d['increment']; print({k: i[k] for k in ('index_ms','upload_ms','migrate_ms','saturate_ms','classification_ms','retrigger','vs_full_classification')})"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-profile --no-throughput2 > $OUT/b0_$i.json 2> $OUT/b0_$i.err || { tail -20 $OUT/b0_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b0_$i.json')); print('plain', d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], d.get('d2h_gbs'))"
done
