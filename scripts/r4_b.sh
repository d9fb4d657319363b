#!/bin/bash
# GPU session (scripts/r4_b.sh TAG): partition tests on the new partitioned path (base links,
# routed exchange), ×2 G3 partition diagnostics on the round-3 library and on the new one, and the
# bench's 2-rank exchange rehearsal (host transport).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_partition.py tests/test_xproc.py > $OUT/part.log 2>&1
rc=$?; tail -4 $OUT/part.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/part.log | head -20; exit $rc; }
EL_GPU_LIB=$R/distel_amd/lib/libel_gpu_r3.so timeout -k 10 300 python -u scripts/part_diag.py g3 1.0 2 2 > $OUT/diag_r3.jsonl 2> $OUT/diag_r3.err || { tail -20 $OUT/diag_r3.err; exit 1; }
python scripts/diag_sum.py $OUT/diag_r3.jsonl
timeout -k 10 300 python -u scripts/part_diag.py g3 1.0 2 3 > $OUT/diag.jsonl 2> $OUT/diag.err || { tail -20 $OUT/diag.err; exit 1; }
python scripts/diag_sum.py $OUT/diag.jsonl
EL_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --transport host --steps 3 --warmup 1 --no-cpu --no-profile > $OUT/b2.json 2> $OUT/b2.err || { tail -20 $OUT/b2.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b2.json')); print({k: d[k] for k in ('ms_per_step','init_ms','saturate_ms','supersteps')}, d['exchange'], d['copies'])"
