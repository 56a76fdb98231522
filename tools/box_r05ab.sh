#!/bin/bash
# Round 5: fused multiply-adds also in sym_err and the relationship estimates.
# The check build, parity, config 3 and config 5 A/B against r05x.
set -o pipefail
TAG=${1:-r05ab}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_bound.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|Error|violat" $OUT/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
MH_AB_REPS=3 MH_AB_CFGS="64,65536,1000,3" bash tools/box_abn.sh $TAG/ab main r05aa || exit 1
