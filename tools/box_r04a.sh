#!/bin/bash
# Round 4, first GPU call: smoke, the numerics edges and one exhaustive quarter of each 32-bit
# probe domain, then an A/B of the shared-math build against HEAD~ (ablate/libmhgpu_head.so) at
# configs 2, 3 and 5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04a; mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_math.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "edges or bm_log-0 or bm_sincos-0 or cos_f32-0 or cos_f32-3 or atan2_room or exp_accept" \
    -W always::UserWarning > $OUT/pytest_math.log 2>&1 || { tail -30 $OUT/pytest_math.log; exit 1; }
grep -E "passed|failed|MathReport" $OUT/pytest_math.log | tail -12
timeout -k 10 300 python -u -m pytest tests/test_c_harness.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_c.log 2>&1 || { tail -30 $OUT/pytest_c.log; exit 1; }
tail -1 $OUT/pytest_c.log
MH_AB_REPS=2 MH_AB_CFGS="64,65536,1000,3 8,1024,2000,4 256,32768,1000,1" bash tools/box_abn.sh r04a/ab head main
