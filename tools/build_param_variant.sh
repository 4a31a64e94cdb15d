#!/bin/bash
# Diagnostic parametric-kernel variants: tools/build_param_variant.sh <name> <extra hipcc flags...>
# compiles csrc/cbn_param.hip with the flags and links it with the main build's
# cbn_infer.o / cbn_direct.o -> continuousbayesiannetwork_amd/libcbn_amd_<name>.so
# (e.g. -DCBN_WPE_LIN=6, -DCBN_MULROW_GROUP=0; SRC= another cbn_param.hip).
set -e
cd "$(dirname "$0")/.."
name=$1; shift
out=continuousbayesiannetwork_amd/libcbn_amd_$name.so
tmp=$(mktemp -d)
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -mcode-object-version=5 -mllvm -amdgpu-kernarg-preload-count=16 -Wno-unused-result -I include"
C=continuousbayesiannetwork_amd/csrc
/opt/rocm/bin/hipcc $F "$@" -c -o $tmp/p.o ${SRC:-$C/cbn_param.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $C/cbn_infer.o $tmp/p.o $C/cbn_direct.o
rm -rf $tmp
echo "built $out"
