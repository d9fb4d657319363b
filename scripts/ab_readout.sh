cd $GRAFT_REPO_ROOT
for w in g3 g3x; do
for m in 0 1; do
  if [ $m = 1 ]; then export EL_NO_READOUT=1; else unset EL_NO_READOUT; fi
  timeout -k 10 300 python bench.py --workload $w --no-cpu --no-profile --steps 10 --warmup 3 > gpurun_out/ab_$w$m.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_$w$m.json')); print('$w noreadout=$m', d['ms_per_step'], 'sat', d['saturate_ms'], 'copy', d['copyback_ms'])"
done; done
