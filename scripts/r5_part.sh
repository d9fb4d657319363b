#!/bin/bash
# GPU session (scripts/r5_part.sh TAG): the partitioned path on one GPU — the partition tests
# (full-size strong scaling included), aligned ×2 and unaligned strong-2 diagnostics, a one-rank
# RCCL bench of both partitioned legs on the system HIP runtime, and the N = 2 bench rehearsed
# with two ranks over gloo (host transport).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_partition.py tests/test_xproc.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python -u scripts/part_diag.py g3 1.0 2 2 weak > $OUT/weak2.jsonl 2> $OUT/weak2.err || { tail -20 $OUT/weak2.err; exit 1; }
timeout -k 10 300 python -u scripts/part_diag.py g3 1.0 2 2 strong > $OUT/strong2.jsonl 2> $OUT/strong2.err || { tail -20 $OUT/strong2.err; exit 1; }
timeout -k 10 300 python bench.py --partition exchange --scaling strong --steps 5 --warmup 2 --no-cpu --no-profile > $OUT/b1x.json 2> $OUT/b1x.err || { tail -20 $OUT/b1x.err; exit 1; }
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --transport host --steps 3 --warmup 1 --no-cpu --no-profile > $OUT/b2.json 2> $OUT/b2.err || { tail -20 $OUT/b2.err; exit 1; }
python - <<PY
import json
for f in ("weak2", "strong2"):
    for l in open("$OUT/%s.jsonl" % f):
        d = json.loads(l)
        if d["leg"] in ("digest", "load"): print(f, d); continue
        if "ranks" in d: print(f, d["step"], d["wall_ms"], d["derived"], [(r["supersteps"], r["init_ms"], r["saturate_ms"], r["exchange_bytes"]) for r in d["ranks"]])
        else: print(f, d["leg"], d["step"], d["supersteps"], d["init_ms"], d["saturate_ms"])
for f in ("b1x", "b2"):
    d = json.loads(open("$OUT/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["scaling"], d.get("hip_runtime"), {k: d.get(k) for k in ("copies", "exchange", "strong")})
PY
