#!/bin/bash
# Timing/probe variants of the full-evaluation kernel only: mh_chain.hip compiled with extra
# defines, linked with the product build's other objects (build/*.o from __graft_entry__.build()).
#   tools/build_chain_variant.sh <name> <-Ddefines...>   ->  abvar/libmhgpu_<name>.so
# ($MH_CHAIN_SRC: an edited copy of mh_chain.hip to compile instead)
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p abvar build/var
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -mllvm -disable-machine-licm -Wno-unused-result"
/opt/rocm/bin/hipcc $F -Imetropolis-hastings-gpgpu_amd/csrc "$@" -c ${MH_CHAIN_SRC:-metropolis-hastings-gpgpu_amd/csrc/mh_chain.hip} -o build/var/chain_$NAME.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC build/var/chain_$NAME.o build/mh_chain_xw.hip.o \
  build/mh_chain_best.hip.o build/mh_delta.hip.o build/mh_spec.hip.o build/mh_abi.cpp.o -o abvar/libmhgpu_$NAME.so
