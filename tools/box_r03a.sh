#!/bin/bash
# On the GPU box: the GPU suite and the driver-shaped bench (with its end-to-end leg) on this
# build, the end-to-end leg with pageable (staged) downloads for the A/B, then the fault
# experiment (tools/box_fault3.sh; may stop at a fault, so it runs last).
set -o pipefail
TAG=${1:-r03a}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('value', d['value'], 'e2e', d['e2e'])"
MH_DOWNLOAD_PAGEABLE=1 timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_pageable.json 2>&1 || { tail -5 $OUT/bench_pageable.json; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_pageable.json').read().strip().splitlines()[-1]); print('pageable e2e', d['e2e'])"
bash tools/box_fault3.sh $TAG/fault3
