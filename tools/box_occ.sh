#!/bin/bash
# On the GPU box: chain-steps/s against resident chains per CU (one launch round each), to see
# how far the step kernels are latency-bound.   tools/box_occ.sh <tag>
set -o pipefail
TAG=${1:-occ}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
run() {  # objects chains iters steps
  timeout -k 10 120 python bench.py --no-cpu-baseline --objects $1 --chains $2 --iters $3 \
      --steps $4 --warmup 1 > $OUT/b_$1_$2.json 2> $OUT/b_$1_$2.err || { tail -5 $OUT/b_$1_$2.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/b_$1_$2.json').read().strip().splitlines()[-1]); print('N=$1 chains=$2 value=%.4g ms/launch=%.2f' % (d['value'], d['kernel_ms_per_launch']))"
}
for c in 1024 2048 3072 4096 8192 16384; do run 64 $c 1000 3 || exit 1; done
for c in 256 512 768 1024 1280 2560; do run 256 $c 300 2 || exit 1; done
