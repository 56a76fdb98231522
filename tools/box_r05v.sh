#!/bin/bash
# Round 5: the incremental kernel with the DPP leader maximum and the DPP double sums (wave_dsum)
# (mh_common.h). Parity (the incremental paths), the check build, config 5 A/B.
set -o pipefail
TAG=${1:-r05v}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_bound.py "tests/test_gpu_configs.py::test_every_chain_short" \
    "tests/test_gpu_configs.py::test_incremental_list_overflow_windows" \
    tests/test_gpu_parity.py -m gpu > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|Error|violat" $OUT/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
MH_AB_REPS=3 MH_AB_CFGS="256,32768,1000,2" bash tools/box_abn.sh $TAG/ab main r05t || exit 1
