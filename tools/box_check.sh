#!/bin/bash
# On the GPU box (via gpurun): the GPU test suite, then a short config-3 bench, then config 2
# at each lanes-per-chain shape.   tools/box_check.sh <tag>
set -o pipefail
TAG=${1:-check}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -40 gpurun_out/$TAG/pytest_gpu.log
[ $rc -le 1 ] || { echo "pytest ended with $rc: stopping"; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 \
    > gpurun_out/$TAG/bench64.json 2> gpurun_out/$TAG/bench64.err || { tail -5 gpurun_out/$TAG/bench64.err; exit 1; }
tail -1 gpurun_out/$TAG/bench64.json
for L in 8 16 32 64; do
  MH_LANES=$L timeout -k 10 120 python bench.py --objects 8 --chains 1024 --iters 1000 --steps 5 \
      --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/c2_L$L.json 2> gpurun_out/$TAG/c2_L$L.err \
      || { tail -5 gpurun_out/$TAG/c2_L$L.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/$TAG/c2_L$L.json').read().strip().splitlines()[-1]); print('config2 L=$L value=%.4g ms/launch=%.2f' % (d['value'], d['kernel_ms_per_launch']))"
done
exit $rc
