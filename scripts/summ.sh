#!/bin/bash
# Summarise a gpu session's bench JSON lines: scripts/summ.sh TAG
cd ${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out
for f in $1/bench.json ${1}x/bench_g5.json ${1}x/bench_g3.json ${1}x/bench_g1.json; do
  [ -f $f ] || continue
  python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['ms_per_step'], round(d['value']/1e6,1), 'M/s steps', d['supersteps'], d['roofline']['kernel'], d['roofline']['frac'], 'parity', d['cpu_baseline'] and d['cpu_baseline']['parity_derived_equal'])"
done
grep -h "passed\|failed" $1/pytest_gpu.log 2>/dev/null | tail -1
