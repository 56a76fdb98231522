#!/bin/bash
# Config-2 (N = 8, 1,024 chains) A/B of step-kernel variants: product vs abvar/libmhgpu_<v>.so,
# alternated twice.   tools/box_ab_n8.sh <tag> <variant>...
set -o pipefail
TAG=${1:-ab8}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
  for V in 0 "$@"; do
    if [ "$V" = 0 ]; then LIB=metropolis-hastings-gpgpu_amd/libmhgpu.so; else LIB=abvar/libmhgpu_$V.so; fi
    MH_LIB=$LIB timeout -k 10 200 python bench.py --objects 8 --chains 1024 --iters 2000 --steps 4 --warmup 1 \
        --no-cpu-baseline --e2e-iters 0 > $OUT/bench_${V}_$rep.json 2> $OUT/bench_${V}_$rep.err || { tail -5 $OUT/bench_${V}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/bench_${V}_$rep.json').read().strip().splitlines()[-1]); print('$V rep $rep value=%.4g ms/launch=%.3f mean=%.8g' % (d['value'], d['kernel_ms_per_launch'], d['mean_final_cost']))"
  done
done
