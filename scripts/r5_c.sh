#!/bin/bash
# GPU session (scripts/r5_c.sh TAG): copy-back tail diagnostics (engines one after another in one
# process), the strong-2 exchange rounds traced, the N = 1 bench with both partitioned legs, and the
# N = 2 rehearsal over gloo.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/tail_diag.py g3 6 whole whole part1 rccl1 whole > $OUT/tail.jsonl 2> $OUT/tail.err || { tail -20 $OUT/tail.err; exit 1; }
cat $OUT/tail.jsonl
EL_TRACE_XCHG=1 timeout -k 10 300 python -u scripts/part_diag.py g3 1.0 2 2 strong > $OUT/strong2.jsonl 2> $OUT/strong2.err || { tail -20 $OUT/strong2.err; exit 1; }
grep "rank 0" $OUT/strong2.err | tail -22
timeout -k 10 300 python bench.py --partition exchange --scaling strong --steps 5 --warmup 2 --no-cpu --no-profile > $OUT/b1x.json 2> $OUT/b1x.err || { tail -20 $OUT/b1x.err; exit 1; }
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --transport host --steps 3 --warmup 1 --no-cpu --no-profile > $OUT/b2.json 2> $OUT/b2.err || { tail -20 $OUT/b2.err; exit 1; }
python - <<PY
import json
for l in open("$OUT/strong2.jsonl"):
    d = json.loads(l)
    if "ranks" in d: print("strong2", d["step"], d["wall_ms"], d["derived"], [(r["supersteps"], r["init_ms"], r["saturate_ms"], r["tail_ms"], r["exchange_bytes"]) for r in d["ranks"]])
for f in ("b1x", "b2"):
    d = json.loads(open("$OUT/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["scaling"], {k: d.get(k) for k in ("copies", "exchange", "strong")})
PY
