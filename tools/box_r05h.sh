#!/bin/bash
# Round 5: speculative kernel v5 (Box-Muller pairs computed per record, words-only window).
set -o pipefail
TAG=${1:-r05h}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_spec.py "tests/test_gpu_configs.py::test_config2_full_length" \
    "tests/test_gpu_configs.py::test_accept_draw_one_rejects_uphill" -m gpu > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|forked|Error" $OUT/pytest.log | tail -4; [ $rc -eq 0 ] || exit $rc
MH_AB_REPS=3 MH_AB_CFGS="8,1024,2000,4" bash tools/box_abn.sh $TAG/ab main r04 || exit 1
for CH in 24576 32768; do
  for SPEC in 1 0; do
    MH_SPEC=$SPEC timeout -k 10 120 python bench.py --objects 8 --chains $CH --iters 2000 --steps 4 \
        --warmup 1 --no-cpu-baseline --e2e-iters 0 > $OUT/spec${SPEC}_$CH.json 2> $OUT/spec${SPEC}_$CH.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/spec${SPEC}_$CH.json').read().strip().splitlines()[-1]); print('MH_SPEC=$SPEC N=8 $CH chains value=%.4g ms/launch=%.3f kernel=%s resident/CU=%s' % (d['value'], d['kernel_ms_per_launch'], d['config'].get('step_kernel'), d['config'].get('resident_chains_per_cu')))"
  done
done
if [ -f ablate/libmhgpu_stamps.so ]; then
  MH_SPEC=1 timeout -k 10 120 python tools/stamps.py 8 1024 2000 > $OUT/stamps_spec_n8.txt 2>&1 || { tail -5 $OUT/stamps_spec_n8.txt; exit 1; }
  cat $OUT/stamps_spec_n8.txt
fi
