#!/bin/bash
# Round 5: config 3's scratch (the proposal's costs and the VisualBalance products to LDS at
# once: 120 -> 52 B per lane). Parity and the check build, A/B against r05o, a PMC pass.
set -o pipefail
TAG=${1:-r05p}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_bound.py "tests/test_gpu_configs.py::test_every_chain_short" \
    tests/test_gpu_parity.py -m gpu > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|Error|violat" $OUT/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
MH_AB_REPS=3 MH_AB_CFGS="64,65536,1000,3" bash tools/box_abn.sh $TAG/ab main r05o || exit 1
bash tools/profile_box.sh $TAG/n64 --steps 3 --warmup 1 --iters 1000 --no-cpu-baseline --e2e-iters 0 || exit 1
python tools/pmc_summary.py $OUT/n64 --kernel "mh_kernel<64, 1, 1>" --chains 65536 --json $OUT/pmc_n64.json \
    --profile profiles/${TAG}_pmc_step_kernel_n64.txt > $OUT/pmc_n64.txt || exit 1
grep -hE "hbm_bytes|fetch|write|valu_issue|insts_per|duration|wait_inst" $OUT/pmc_n64.txt
