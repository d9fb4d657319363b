#!/bin/bash
# Build distel_amd/lib/variants/libel_gpu_TAG.so from the library sources of git revision REV
# (A/B of a change against the commit before it; selected at run time by EL_LIB_VARIANT=TAG).
# Usage: scripts/build_rev.sh TAG REV [-DFLAG=V ...]
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; REV=$2; shift 2
T=$(mktemp -d)
git -C $R archive $REV distel_amd/csrc include | tar -x -C $T
mkdir -p $R/distel_amd/lib/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wl,--no-undefined "$@" -I$T/include \
  -o $R/distel_amd/lib/variants/libel_gpu_$TAG.so $T/distel_amd/csrc/el_gpu.hip $T/distel_amd/csrc/el_rows.hip \
  $T/distel_amd/csrc/el_closure.hip $T/distel_amd/csrc/el_stream.hip $T/distel_amd/csrc/el_index.cpp
rm -rf $T
