#!/bin/bash
# GPU session (scripts/r5_final2.sh TAG): the partitioned path's record on the final source —
# strong scaling of one G3 on 2 and 4 row partitions (LOCAL transport, one process) with the
# per-superstep exchange records (EL_TRACE_XCHG) and device bytes per structure (EL_TRACE_MEM);
# ×8 of G3 at 50 % on 8 aligned partitions (configs[3] shape) with EL_TRACE_MEM; the N = 2 bench
# rehearsed with two ranks over gloo (host transport) on one GPU; and the same two ranks each
# under its own rocprofv3 kernel trace (ranks started by hand, no launcher under the profiler)
# to show which kernels run beside the supersteps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for k in 2 4; do
  EL_TRACE_XCHG=1 EL_TRACE_MEM=1 timeout -k 10 400 python -u scripts/part_diag.py g3 1.0 $k 2 strong > $OUT/strong$k.jsonl 2> $OUT/strong$k.err || { tail -20 $OUT/strong$k.err; exit 1; }
done
EL_TRACE_MEM=1 timeout -k 10 400 python -u scripts/part_diag.py g3 0.5 8 1 weak > $OUT/weak8_half.jsonl 2> $OUT/weak8_half.err || { tail -20 $OUT/weak8_half.err; exit 1; }
grep "^mem rank 0" -A14 $OUT/weak8_half.err | head -16
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --transport host --steps 3 --warmup 1 --no-cpu --no-profile > $OUT/b2.json 2> $OUT/b2.err || { tail -20 $OUT/b2.err; exit 1; }
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --scaling strong --transport host --steps 3 --warmup 1 --no-cpu --no-profile > $OUT/b2s.json 2> $OUT/b2s.err || { tail -20 $OUT/b2s.err; exit 1; }
pids=()
for r in 0 1; do
  (cd /tmp && RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 \
    timeout -k 10 500 rocprofv3 --kernel-trace -d $OUT/rk$r -o tr -- python3 $R/bench.py --gpus 2 --transport host --steps 2 --warmup 1 --no-cpu --no-profile > $OUT/rk$r.json 2> $OUT/rk$r.err) &
  pids+=($!)
done
wait ${pids[0]} || { tail -20 $OUT/rk0.err; exit 1; }
wait ${pids[1]} || { tail -20 $OUT/rk1.err; exit 1; }
for r in 0 1; do python3 scripts/rpd_stats.py "$OUT/rk$r/tr_results.db" > $OUT/rk${r}_stats.csv && head -12 $OUT/rk${r}_stats.csv; done
python - <<PY
import json
for f in ("strong2", "strong4", "weak8_half"):
    for l in open("$OUT/%s.jsonl" % f):
        d = json.loads(l)
        if d["leg"] in ("digest", "load"): print(f, d); continue
        if "ranks" in d: print(f, d["step"], d["wall_ms"], d["derived"], [(r["supersteps"], r["init_ms"], r["saturate_ms"], r["exchange_bytes"]) for r in d["ranks"]])
        else: print(f, d["leg"], d["step"], d["supersteps"], d["init_ms"], d["saturate_ms"])
for f in ("b2", "b2s"):
    d = json.loads(open("$OUT/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["scaling"], d.get("hip_runtime"), {k: d.get(k) for k in ("copies", "exchange", "strong")})
PY
