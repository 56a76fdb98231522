#!/bin/bash
# Round 5: tree speculation (mh_spec.hip). The speculative kernel's parity cases and config 2 in
# full, then an A/B against round 4's library at config 2 (1,024 chains) and the speculative /
# full-evaluation choice at 2,048 chains (the cutoff n_chains <= 8 x CUs).
set -o pipefail
TAG=${1:-r05b}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_spec.py "tests/test_gpu_configs.py::test_config2_full_length" \
    "tests/test_gpu_configs.py::test_index_n_pick_redrawn" \
    "tests/test_gpu_configs.py::test_accept_draw_one_rejects_uphill" \
    "tests/test_gpu_configs.py::test_kernelwrapper_pooled_sessions" "tests/test_gpu_configs.py::test_kernelwrapper_mh_devices_sharding" -m gpu > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|ParityReport|forked|Error" $OUT/pytest.log | tail -40; [ $rc -eq 0 ] || exit $rc
MH_AB_REPS=3 MH_AB_CFGS="8,1024,2000,4" bash tools/box_abn.sh $TAG/ab main r04 || exit 1
for SPEC in 1 0; do
  MH_SPEC=$SPEC timeout -k 10 120 python bench.py --objects 8 --chains 2048 --iters 2000 --steps 4 \
      --warmup 1 --no-cpu-baseline --e2e-iters 0 > $OUT/spec${SPEC}_2048.json 2> $OUT/spec${SPEC}_2048.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/spec${SPEC}_2048.json').read().strip().splitlines()[-1]); print('MH_SPEC=$SPEC N=8 2048 chains value=%.4g ms/launch=%.3f kernel=%s' % (d['value'], d['kernel_ms_per_launch'], d['config'].get('step_kernel')))"
done
timeout -k 10 120 python tools/wrapper_overhead.py 10 > $OUT/wrapper_overhead.jsonl 2>&1 || exit 1
cat $OUT/wrapper_overhead.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --hip-trace --stats -d $OUT/prof_wrapper -o wrap -- python tools/wrapper_overhead.py 3 > $OUT/prof_wrapper.log 2>&1 || { tail -5 $OUT/prof_wrapper.log; exit 1; }
find $OUT/prof_wrapper -name "*hip_api_stats.csv" | head -3
