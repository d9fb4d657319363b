#!/bin/bash
# Build distel_amd/lib/variants/libel_gpu_TAG.so with extra compile flags (A/B builds, selected at
# run time by EL_LIB_VARIANT=TAG).  Usage: scripts/build_variant.sh TAG -DFLAG=V ...
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; shift
mkdir -p $R/distel_amd/lib/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wl,--no-undefined "$@" -I$R/include \
  -o $R/distel_amd/lib/variants/libel_gpu_$TAG.so $R/distel_amd/csrc/el_gpu.hip $R/distel_amd/csrc/el_rows.hip \
  $R/distel_amd/csrc/el_closure.hip $R/distel_amd/csrc/el_stream.hip $R/distel_amd/csrc/el_index.cpp
