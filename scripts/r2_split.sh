#!/bin/bash
# Kernel trace of G3 with k_expand split per role / rule group (EL_SPLIT_EXPAND=2), serial.
set -o pipefail
TAG=${1:-split}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
EL_SPLIT_EXPAND=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --inflight 1 --no-cpu --no-profile --steps 2 --warmup 1 > $OUT/prof.log 2>&1
