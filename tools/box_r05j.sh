#!/bin/bash
# Round 5: the incremental kernel's replay with full-length typed zero streams (round 4's code
# shape, no punning): parity and config 5 against round 4.
set -o pipefail
TAG=${1:-r05j}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    "tests/test_gpu_configs.py::test_every_chain_short" "tests/test_gpu_configs.py::test_incremental_list_overflow_windows" \
    "tests/test_gpu_parity.py::test_running_costs_equal_fresh_evaluation" -m gpu > $OUT/pytest_delta.log 2>&1
rc=$?; grep -E "passed|failed|forked" $OUT/pytest_delta.log | tail -8; [ $rc -eq 0 ] || exit $rc
MH_AB_REPS=3 MH_AB_CFGS="256,32768,1000,2" bash tools/box_abn.sh $TAG/ab5 main r04 || exit 1
python bench.py --objects 256 --chains 32768 --iters 1000 --steps 2 --warmup 1 --no-cpu-baseline --e2e-iters 0 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('resident/CU', d['config']['resident_chains_per_cu'])"
