#!/bin/bash
# Round 4: per-phase cycles of the speculative kernel and of the few-chains step kernel at
# config 2, then an A/B of the shared math inlined / out of line (MH_MATH_OOL masks) at configs
# 3, 2 (non-speculative) and 5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04e; mkdir -p $OUT
MH_SPEC=1 timeout -k 10 120 python -u tools/stamps.py 8 1024 2000 > $OUT/stamps_spec.txt 2>&1; rc=$?; cat $OUT/stamps_spec.txt; [ $rc = 0 ] || exit 1
MH_SPEC=0 timeout -k 10 120 python -u tools/stamps.py 8 1024 2000 > $OUT/stamps_few.txt 2>&1; rc=$?; cat $OUT/stamps_few.txt; [ $rc = 0 ] || exit 1
export MH_SPEC=0
MH_AB_REPS=2 MH_AB_CFGS="64,65536,1000,3 8,1024,2000,4 256,32768,1000,1" bash tools/box_abn.sh r04e/ab head ool0 ool1 ool5 main
