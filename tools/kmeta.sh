#!/bin/bash
# Kernel resource metadata (LDS, scratch, SGPR/VGPR) of one HIP source for gfx950:
#   tools/kmeta.sh snf4j_amd/csrc/inflate.hip [name-filter]
src=$1; filt=${2:-.}
tmp=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -disable-promote-alloca-to-lds --cuda-device-only \
  -c "$src" -o "$tmp/b.o" $KMETA_FLAGS || exit 1
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$tmp/b.o" \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$tmp/d.o" || exit 1
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$tmp/d.o" |
  grep -E "^\s+\.name:|\.vgpr_count|\.sgpr_count|group_segment_fixed_size|private_segment_fixed_size" |
  paste - - - - - | sed 's/  */ /g' | grep -E "$filt"
rm -rf "$tmp"
