#!/bin/bash
# A/B of copy-back variants: read-out chunk size on G3; small-S path (direct sorts vs DMA) on G5 / G2.
cd ${GRAFT_REPO_ROOT:-.}
run() {  # tag workload env...
  local tag=$1 w=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $w --no-cpu --no-profile --steps 10 --warmup 3 > gpurun_out/abc_$tag.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/abc_$tag.json')); print('$tag', d['ms_per_step'], 'sat', d['saturate_ms'], 'copy', d['copyback_ms'], 'derived', d['derived_axioms'])"
}
run g3_c32 g3 EL_READOUT_CHUNK_MB=32
run g3_c64 g3 EL_READOUT_CHUNK_MB=64
run g3_c128 g3 EL_READOUT_CHUNK_MB=128
run g5_direct g5 X=1
run g5_sdma g5 EL_S_DMA=1
run g2_direct g2 X=1
run g2_sdma g2 EL_S_DMA=1
