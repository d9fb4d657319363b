#!/bin/bash
# GPU session (scripts/r5_part_co.sh TAG): the whole GPU suite, then the partitioned path with
# the column order on and off (EL_COLUMN_ORDER=0): ×2 aligned (weak) and one G3 on 2 ranks
# (strong), LOCAL transport in one process (scripts/part_diag.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
for mode in weak strong; do
  for v in def id; do
    E=""; [ $v = id ] && E="EL_COLUMN_ORDER=0"
    env $E timeout -k 10 300 python -u scripts/part_diag.py g3 1.0 2 3 $mode > $OUT/${mode}_$v.jsonl 2> $OUT/${mode}_$v.err || { tail -20 $OUT/${mode}_$v.err; exit 1; }
    python3 - <<PY
import json
for l in open("$OUT/${mode}_$v.jsonl"):
    d = json.loads(l)
    if "ranks" in d and d["step"] > 0: print("$mode $v", d["step"], d["wall_ms"], d["derived"], [(r["supersteps"], r["init_ms"], r["saturate_ms"]) for r in d["ranks"]])
    if d.get("leg") == "digest": print("$mode $v digest equal", d["equal"])
PY
  done
done
