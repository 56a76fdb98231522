#!/bin/bash
# On the GPU box: stamps of configs 3, 5, 2 (ablate/libmhgpu_stamps.so), then the bound check and
# the config-3 / config-5 bench lines of this build (the GPU suite is left to the next call).
set -o pipefail
TAG=${1:-r03i}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/box_stamps.sh $TAG/stamps || exit 1
timeout -k 10 600 python -u tools/bound_check.py > $OUT/bound_check.txt 2>&1 || { cat $OUT/bound_check.txt; exit 1; }
cut -c1-200 $OUT/bound_check.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_n64.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
timeout -k 10 300 python bench.py --objects 256 --chains 32768 --iters 1000 --steps 8 --warmup 1 --no-cpu-baseline --e2e-iters 0 > $OUT/bench_n256.json 2>> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
for f in $OUT/bench_n64.json $OUT/bench_n256.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['kernel_ms_per_launch'], d['mean_final_cost'])"; done
