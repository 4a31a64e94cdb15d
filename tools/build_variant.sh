#!/bin/bash
# Diagnostic library variants: tools/build_variant.sh <name> <extra hipcc flags...>
# e.g. tools/build_variant.sh stamps -DCBN_STAMPS -> continuousbayesiannetwork_amd/libcbn_amd_stamps.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
out=continuousbayesiannetwork_amd/libcbn_amd_$name.so
tmp=$(mktemp -d)
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -mcode-object-version=5 -mllvm -amdgpu-kernarg-preload-count=16 -Wno-unused-result -I include"
/opt/rocm/bin/hipcc $F "$@" -c -o $tmp/a.o continuousbayesiannetwork_amd/csrc/cbn_infer.hip &
/opt/rocm/bin/hipcc $F "$@" -c -o $tmp/b.o continuousbayesiannetwork_amd/csrc/cbn_param.hip &
/opt/rocm/bin/hipcc $F "$@" -c -o $tmp/c.o continuousbayesiannetwork_amd/csrc/cbn_direct.hip &
wait %1 && wait %2 && wait %3
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $tmp/a.o $tmp/b.o $tmp/c.o
rm -rf $tmp
echo "built $out"
