#!/bin/bash
# GPU session (scripts/r4_a.sh TAG): the row-partitioned path on one GPU — ×2 of G3 on 2 partitions
# in one process (LOCAL transport, HIP-event kernel tables), the same under rocprofv3 kernel trace,
# and the bench's 2-rank exchange rehearsal (host transport).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/part_diag.py g3 1.0 2 3 > $OUT/diag.jsonl 2> $OUT/diag.err || { tail -20 $OUT/diag.err; exit 1; }
python - <<'EOF' $OUT/diag.jsonl
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    if d["leg"] == "whole":
        print("whole", d["step"], d["init_ms"], d["saturate_ms"], d["supersteps"])
    elif d["leg"] == "load":
        print("load", d["s"])
    else:
        print(d["leg"], d["step"], d["wall_ms"], [(r["init_ms"], r["saturate_ms"], r["supersteps"], r["exchange_bytes"]) for r in d["ranks"]])
EOF
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o diag -- python3 $R/scripts/part_diag.py g3 1.0 2 2 > $OUT/prof.log 2>&1) || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
EL_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --transport host --steps 3 --warmup 1 --no-cpu --no-profile > $OUT/b2.json 2> $OUT/b2.err || { tail -20 $OUT/b2.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b2.json')); print({k: d[k] for k in ('ms_per_step','init_ms','saturate_ms','supersteps')}, d['copies'])"
