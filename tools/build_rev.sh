#!/bin/bash
# Builds the product library of a git revision into abvar/libmhgpu_<name>.so (A/B timing
# against the working tree in one GPU call).   tools/build_rev.sh <rev> <name>
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=$2
T=$(mktemp -d)
mkdir -p $T/metropolis-hastings-gpgpu_amd/csrc $T/include abvar
for f in $(git ls-tree --name-only $REV metropolis-hastings-gpgpu_amd/csrc/) include/mh_kernel.h; do
  git show $REV:$f > $T/$f
done
C=$T/metropolis-hastings-gpgpu_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -mllvm -disable-machine-licm \
  -Wno-unused-result $C/mh_chain.hip $C/mh_chain_xw.hip $C/mh_chain_best.hip $C/mh_delta.hip \
  $(test -f $C/mh_spec.hip && echo $C/mh_spec.hip) $C/mh_abi.cpp \
  -o abvar/libmhgpu_$NAME.so
rm -rf $T
