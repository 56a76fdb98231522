#!/bin/bash
# Round 4: the speculative kernel's parity tests, then an A/B at configs 3, 2 and 5 of HEAD~
# (OCML math), "inl" (shared math inlined) and the working tree (shared math, rare paths out of
# line; the speculative kernel at config 2).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04c; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider -W always::UserWarning > $OUT/pytest_spec.log 2>&1 || { tail -40 $OUT/pytest_spec.log; exit 1; }
grep -E "passed|failed|ParityReport" $OUT/pytest_spec.log | tail -14
MH_AB_REPS=2 MH_AB_CFGS="64,65536,1000,3 8,1024,2000,4 256,32768,1000,1" bash tools/box_abn.sh r04c/ab head inl main
bash tools/box_fault4.sh r04c/fault4
