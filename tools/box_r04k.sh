#!/bin/bash
# Round 4: the one-division atan2 (mh_atan_ratio): device == oracle on the atan2 probes, parity of
# every step kernel, then an A/B against the previous commit (two-division atan2) at configs 3,
# 2 and 5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r04k}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_math.py tests/test_gpu_parity.py tests/test_gpu_spec.py -m gpu -x -v \
    --timeout 300 --timeout-method thread -p no:cacheprovider -W always::UserWarning -k "atan2 or parity or spec or incremental or full" \
    > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
grep -E "passed|failed" $OUT/pytest.log | tail -2
grep -E "MathReport probe atan2" $OUT/pytest.log | sed 's/.*MathReport: //' | sort -u
MH_AB_REPS=2 MH_AB_CFGS="64,65536,1000,3 8,1024,2000,4 256,32768,1000,1" bash tools/box_abn.sh ${1:-r04k}/ab prev main
