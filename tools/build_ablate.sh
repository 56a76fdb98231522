#!/bin/bash
# Timing-only variants of libmhgpu.so with phases compiled out (MH_ABLATE bitmask):
#   1 symmetry rows, 2 per-object atan2/cos, 4 ordered sums, 8 SurfaceArea/Clearance pairs,
#   16 PairWise/Angle, 32 Box-Muller. Results are WRONG by construction; only time matters.
# `check` validates every computed index in the full-evaluation kernel and records the first
# violation (mh_debug_check) instead of accessing it; `countscheck` is the counting build with it.
# `stamps` builds the per-phase cycle-stamp diagnostic (tools/stamps.py) instead; `dblK`
# runs phase bit K twice with identical results (cost probe: the trajectory is unchanged).
set -e
cd "$(dirname "$0")/.."
mkdir -p abvar
C=metropolis-hastings-gpgpu_amd/csrc
for M in "$@"; do
  case "$M" in
    stamps) DEF=-DMH_STAMPS=1 ;;
    counts) DEF=-DMH_STAMPS=2 ;;
    countscheck) DEF="-DMH_STAMPS=2 -DMH_CHECK=1" ;;
    check) DEF=-DMH_CHECK=1 ;;
    countsinl) DEF="-DMH_STAMPS=2 -DMH_EVAL_INLINE=1" ;;
    noinl) DEF=-DMH_EVAL_INLINE=-1 ;;
    specdbg) DEF=-DMH_SPEC_DEBUG=1 ;;
    ocml*) DEF=-DMH_ABLATE_OCML=${M#ocml} ;;
    ool*) DEF=-DMH_MATH_OOL=${M#ool} ;;
    wpe*) DEF=-DMH_WAVES_PER_EU=${M#wpe} ;;
    dbl*) DEF=-DMH_DOUBLE=${M#dbl} ;;
    *) DEF=-DMH_ABLATE=$M ;;
  esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -mllvm -disable-machine-licm \
    -Wno-unused-result $DEF $C/mh_chain.hip $C/mh_chain_xw.hip $C/mh_chain_best.hip $C/mh_delta.hip $C/mh_spec.hip \
    $C/mh_abi.cpp -o abvar/libmhgpu_$M.so &
done
wait
