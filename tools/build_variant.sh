#!/bin/bash
# A/B build: recompile ONE translation unit of the library with extra flags and
# link it with the product objects of liblcb_amd/build into
# ab_builds/<name>/liblcb_hash_gpu.so (select it on the box with
# LCB_HASH_GPU_LIB=ab_builds/<name>/liblcb_hash_gpu.so).
#   tools/build_variant.sh <name> <tu, e.g. gost_kernels.hip> [hipcc flags...]
# SRC=<dir> compiles the unit from another source tree (e.g. a git checkout
# of an earlier revision's liblcb_amd/csrc, for a same-box A/B).
set -e
name=$1; tu=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
out=$ROOT/ab_builds/$name
mkdir -p "$out"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" \
    -c -o "$out/$tu.o" "${SRC:-$ROOT/liblcb_amd/csrc}/$tu"
objs=$(ls "$ROOT"/liblcb_amd/build/*.o | grep -v "/$tu.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$out/liblcb_hash_gpu.so" $objs "$out/$tu.o"
python3 "$ROOT/tools/kernel_resources.py" --spills "$out/liblcb_hash_gpu.so" | tail -1
