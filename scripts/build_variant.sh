#!/bin/bash
# A build variant of libwsgpu.so for same-box A/B (scripts/ab_line.sh, ab_lib.sh):
#   scripts/build_variant.sh <tag> <source.hip | path/to/source.hip> <-Dflags...>
# recompiles one source with the extra flags and links it with the in-tree build's
# other objects into snf4j_amd/_ab/libwsgpu_<tag>.so (run the normal build first).
cd "$(dirname "$0")/.."
tag=$1; src=$2; shift 2
mkdir -p snf4j_amd/_ab/obj
path=snf4j_amd/csrc/$src
case "$src" in */*) path=$src ;; esac  # a path: e.g. an earlier revision of a source
obj=snf4j_amd/_ab/obj/${tag}_$(basename "$src" .hip).o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
  -mllvm -disable-promote-alloca-to-lds -Isnf4j_amd/csrc -Iinclude "$@" -c "$path" -o "$obj" || exit 1
objs=$(ls snf4j_amd/_build/*.o | grep -v "/$(basename "$src" .hip).o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "snf4j_amd/_ab/libwsgpu_$tag.so" $objs "$obj" || exit 1
echo "snf4j_amd/_ab/libwsgpu_$tag.so"
