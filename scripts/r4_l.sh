#!/bin/bash
# GPU session (scripts/r4_l.sh TAG [VARIANTS...]): parity tests; a warm-up bench, then G3 A/B of the
# variants given as NAME=ENV pairs (def = no env), two rounds; a kernel trace of the default.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
shift
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/t.log | head -20; exit $rc; }
B="bench.py --no-cpu --no-throughput2 --steps 10 --warmup 3"
timeout -k 10 200 python $B > $OUT/warm.json 2> $OUT/warm.err || { tail $OUT/warm.err; exit 1; }
for rep in 1 2; do
  for kv in def "$@"; do
    v=${kv%%=*}; E=""; [ "$kv" != def ] && E=${kv#*=}
    env $E timeout -k 10 200 python $B > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || { tail $OUT/ab_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python -c "import json; d=json.load(open('$OUT/ab_${v}_$rep.json')); k=d['kernels']; print(d['ms_per_step'], d['init_ms'], d['saturate_ms'], d['copyback_ms'], 'closure', k['k_closure']['ms'], 'init', k['k_init']['ms'], 'commit', k['k_commit']['ms'])")"
  done
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o tr -- python3 $R/bench.py --no-cpu --no-profile --no-throughput2 --steps 10 --warmup 3 > $OUT/tr.json 2> $OUT/tr.err) || { tail $OUT/tr.err; exit 1; }
echo "trace $(python -c "import json; d=json.loads(open('$OUT/tr.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['init_ms'], d['saturate_ms'])")"
python3 scripts/rpd_stats.py $OUT/tr/tr_results.db > $OUT/tr_stats.csv
head -16 $OUT/tr_stats.csv
python3 scripts/steps.py $OUT/tr/tr_results.db 5 > $OUT/tr_steps.txt
head -8 $OUT/tr_steps.txt
