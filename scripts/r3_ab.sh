#!/bin/bash
# G3 bench A/B (scripts/r3_ab.sh TAG LIB_B [rounds]): the built library vs another build (EL_GPU_LIB),
# alternating, one line each (ms per classification, init, saturate).  Optional first step: the
# parity tests of the built library (AB_TESTS=1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
if [ "$AB_TESTS" = "1" ]; then
  timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_workloads.py > $OUT/t.log 2>&1
  rc=$?; tail -1 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
fi
for i in $(seq 1 ${3:-3}); do
  timeout -k 10 200 python bench.py --no-cpu --no-throughput2 --no-profile --steps 5 --warmup 2 > $OUT/a$i.json 2>>$OUT/err || exit 1
  EL_GPU_LIB=$2 timeout -k 10 200 python bench.py --no-cpu --no-throughput2 --no-profile --steps 5 --warmup 2 > $OUT/b$i.json 2>>$OUT/err || exit 1
  python3 -c "import json,sys; [print(f.split('/')[-1], d['ms_per_step'], d['init_ms'], d['saturate_ms']) for f in sys.argv[1:] for d in [json.load(open(f))]]" $OUT/a$i.json $OUT/b$i.json
done
