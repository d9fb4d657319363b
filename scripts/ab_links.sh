#!/bin/bash
# A/B of the link-row copy-back: device sort + DMA (default) vs sorts writing the host buffer.
cd ${GRAFT_REPO_ROOT:-.}
for w in g3 g5 g2; do
for m in 0 1; do
  if [ $m = 1 ]; then export EL_LINKS_DIRECT=1; else unset EL_LINKS_DIRECT; fi
  timeout -k 10 300 python bench.py --workload $w --no-cpu --no-profile --steps 10 --warmup 3 > gpurun_out/abl_$w$m.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/abl_$w$m.json')); print('$w links_direct=$m', d['ms_per_step'], 'sat', d['saturate_ms'], 'copy', d['copyback_ms'])"
done; done
