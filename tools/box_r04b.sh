#!/bin/bash
# Round 4: the full numerics check (every probe, exhaustive / 2^30 samples), then the A/B of the
# shared-math build against HEAD~ (ablate/libmhgpu_head.so) at configs 3, 2 and 5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04b; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_math.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider -W always::UserWarning > $OUT/pytest_math.log 2>&1 || { tail -30 $OUT/pytest_math.log; exit 1; }
grep -E "passed|failed|MathReport probe" $OUT/pytest_math.log | tail -30
MH_AB_REPS=2 MH_AB_CFGS="64,65536,1000,3 8,1024,2000,4 256,32768,1000,1" bash tools/box_abn.sh r04b/ab head main
