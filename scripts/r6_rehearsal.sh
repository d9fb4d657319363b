#!/bin/bash
# GPU session (scripts/r6_rehearsal.sh TAG): the bench's N = 2 command rehearsed on one GPU (two
# ranks, gloo host transport; RCCL refuses two ranks on one card) with the default legs — the
# per-rank roofline of the partitioned leg and rank 0's cpu_baseline included.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
EL_DIST_BACKEND=gloo timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --transport host --steps 3 --warmup 1 > $OUT/b2.json 2> $OUT/b2.err || { tail -20 $OUT/b2.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/b2.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline'], {k: d['cpu_baseline'][k] for k in ('value','cores','kind')})"
