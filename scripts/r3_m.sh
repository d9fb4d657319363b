#!/bin/bash
# GPU session (scripts/r3_m.sh TAG): parity / workload / export tests, then G3 bench A/B of an
# environment knob (ENV_B, e.g. EL_BASE_JOIN=1), alternating, verbose lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_gpu_export.py tests/test_gpu_incremental.py > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu --no-throughput2 --no-profile --steps 5 --warmup 2 > $OUT/a$i.json 2>>$OUT/err || exit 1
  env $ENV_B timeout -k 10 200 python bench.py --no-cpu --no-throughput2 --no-profile --steps 5 --warmup 2 > $OUT/b$i.json 2>>$OUT/err || exit 1
  python3 -c "import json,sys; [print(f, d['ms_per_step'], d['init_ms'], d['saturate_ms']) for f in sys.argv[1:] for d in [json.load(open(f))]]" $OUT/a$i.json $OUT/b$i.json
done
