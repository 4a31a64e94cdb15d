#!/bin/bash
# Diagnostic library variants: tools/build_variant.sh <name> <extra hipcc flags...>
# e.g. tools/build_variant.sh stamps -DCBN_STAMPS -> continuousbayesiannetwork_amd/libcbn_amd_stamps.so
# The diagnostic macros only touch cbn_infer.hip: the parametric and direct
# TUs are linked from the main build's objects when present (build() leaves
# them in csrc/), else compiled here.
set -e
cd "$(dirname "$0")/.."
name=$1; shift
out=continuousbayesiannetwork_amd/libcbn_amd_$name.so
tmp=$(mktemp -d)
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -mcode-object-version=5 -mllvm -amdgpu-kernarg-preload-count=${PRELOAD:-16} -Wno-unused-result -I include"
C=continuousbayesiannetwork_amd/csrc
/opt/rocm/bin/hipcc $F "$@" -c -o $tmp/a.o ${SRC:-$C/cbn_infer.hip}
for t in cbn_param cbn_direct; do
  if [ -f $C/$t.o ] && [ $C/$t.o -nt $C/$t.hip ]; then cp $C/$t.o $tmp/$t.o
  else /opt/rocm/bin/hipcc $F "$@" -c -o $tmp/$t.o $C/$t.hip; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $tmp/a.o $tmp/cbn_param.o $tmp/cbn_direct.o
rm -rf $tmp
echo "built $out"
