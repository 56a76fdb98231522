#!/bin/bash
# Round 5: the speculative kernel with per-window step records, role-sized LDS and the fp32
# Accept screen. Parity (speculative cases, config 2 in full, the accept probe), then timing
# against round 4's library and the speculative / few-chains choice by chain count.
set -o pipefail
TAG=${1:-r05d}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_spec.py "tests/test_gpu_configs.py::test_config2_full_length" \
    "tests/test_gpu_math.py::test_sampled_arguments" "tests/test_gpu_math.py::test_probe_edges" \
    "tests/test_gpu_configs.py::test_accept_draw_one_rejects_uphill" -m gpu > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|ParityReport|MathReport|forked|Error" $OUT/pytest.log | tail -40; [ $rc -eq 0 ] || exit $rc
MH_AB_REPS=3 MH_AB_CFGS="8,1024,2000,4" bash tools/box_abn.sh $TAG/ab main r04 || exit 1
for CH in 1536 1792 2048; do
  for SPEC in 1 0; do
    MH_SPEC=$SPEC timeout -k 10 120 python bench.py --objects 8 --chains $CH --iters 2000 --steps 4 \
        --warmup 1 --no-cpu-baseline --e2e-iters 0 > $OUT/spec${SPEC}_$CH.json 2> $OUT/spec${SPEC}_$CH.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/spec${SPEC}_$CH.json').read().strip().splitlines()[-1]); print('MH_SPEC=$SPEC N=8 $CH chains value=%.4g ms/launch=%.3f kernel=%s resident/CU=%s' % (d['value'], d['kernel_ms_per_launch'], d['config'].get('step_kernel'), d['config'].get('resident_chains_per_cu')))"
  done
done
