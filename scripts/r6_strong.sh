#!/bin/bash
# GPU session (scripts/r6_strong.sh TAG): the strong-scaling partition (one G3 on 2 and 4 ranks,
# rows by ir.balanced_rows) — its full-size digest tests, per-rank tables (part_diag.py strong:
# derived axioms, supersteps, kernel times per rank) and the N = 2 strong bench rehearsal (two
# processes on one GPU, gloo host transport) with the per-rank roofline.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "strong" > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
for k in 2 4; do
  timeout -k 10 400 python -u scripts/part_diag.py g3 1.0 $k 2 strong > $OUT/strong$k.jsonl 2> $OUT/strong$k.err || { tail -20 $OUT/strong$k.err; exit 1; }
  python3 scripts/diag_sum.py $OUT/strong$k.jsonl | tail -6
done
EL_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --scaling strong --transport host --steps 3 --warmup 1 > $OUT/b2s.json 2> $OUT/b2s.err || { tail -20 $OUT/b2s.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/b2s.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['supersteps'], d['roofline']['kernel'], d['roofline']['frac'], d['strong'])"
