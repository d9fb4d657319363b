#!/bin/bash
# GPU session (scripts/r5_inc.sh TAG): incremental classification as a delta — the incremental
# tests, then the bench with a 1 % G3 increment timed beside the full classification.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_incremental.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python bench.py --increment 0.01 --steps 5 --warmup 2 --no-cpu --no-profile --no-throughput2 > $OUT/b1.json 2> $OUT/b1.err || { tail -20 $OUT/b1.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b1.json')); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], d.get('d2h_gbs')); print(json.dumps(d['increment']))"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-profile --no-throughput2 > $OUT/b0_$i.json 2> $OUT/b0_$i.err || { tail -20 $OUT/b0_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b0_$i.json')); print('plain', d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], d.get('d2h_gbs'))"
done
