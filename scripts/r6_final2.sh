#!/bin/bash
# GPU session (scripts/r6_final2.sh TAG): the round's record, part 2 (after r6_final.sh committed
# the PMC summary of the same source) — the default bench line (G3, N = 1, cpu_baseline with the
# whole-G3 one-core run), the lines of the other workloads, the 1 % G3 increment line and the
# N = 2 bench rehearsed on one GPU (two ranks, gloo host transport).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
for w in g1 g2 g5 g3x g3e; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu --steps 10 --warmup 3 > $OUT/b_$w.json 2> $OUT/b_$w.err || { tail $OUT/b_$w.err; exit 1; }
  echo "$w $(python -c "import json; d=json.load(open('$OUT/b_$w.json')); print(d['ms_per_step'], d['value'], d['init_ms'], d['saturate_ms'], d['copyback_ms'])")"
done
timeout -k 10 300 python bench.py --increment 0.01 --steps 5 --warmup 1 --no-cpu --no-profile --no-throughput2 > $OUT/inc.json 2> $OUT/inc.err || { tail $OUT/inc.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/inc.json')); i=d['increment']; print('increment', {k: i[k] for k in ('index_ms','upload_ms','migrate_ms','saturate_ms','classification_ms','retrigger','vs_full_classification')})"
EL_DIST_BACKEND=gloo timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --transport host --steps 3 --warmup 1 > $OUT/b2.json 2> $OUT/b2.err || { tail -20 $OUT/b2.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/b2.json').read().strip().splitlines()[-1]); print('N=2', d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
