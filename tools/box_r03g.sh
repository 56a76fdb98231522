#!/bin/bash
# On the GPU box: the bound's decisions and the fp32 estimates verified (check build), the GPU
# suite, and the bench lines of configs 3, 5 and 2 on this build.
set -o pipefail
TAG=${1:-r03g}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u tools/bound_check.py > $OUT/bound_check.txt 2>&1 || { cat $OUT/bound_check.txt; exit 1; }
cat $OUT/bound_check.txt | cut -c1-200
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_n64.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
timeout -k 10 300 python bench.py --objects 256 --chains 32768 --iters 1000 --steps 8 --warmup 1 --no-cpu-baseline --e2e-iters 0 > $OUT/bench_n256.json 2>> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
timeout -k 10 300 python bench.py --objects 8 --chains 1024 --iters 4000 --steps 5 --warmup 1 --no-cpu-baseline --e2e-iters 0 > $OUT/bench_n8.json 2>> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
for f in $OUT/bench_n64.json $OUT/bench_n256.json $OUT/bench_n8.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['kernel_ms_per_launch'], d['mean_final_cost'])"; done
