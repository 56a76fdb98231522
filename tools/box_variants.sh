#!/bin/bash
# On the GPU box: the config-3 (and optionally config-5) bench for each library variant under
# ablate/ (timing only).   tools/box_variants.sh <tag> <variant>... (e.g. wpe5 wpe6; "main" =
# the product library)
set -o pipefail
TAG=${1:-variants}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
for V in "$@"; do
  if [ "$V" = main ]; then unset MH_LIB; else export MH_LIB=abvar/libmhgpu_$V.so; fi
  for CFG in ${MH_VARIANT_CFGS:-64,65536,1000,5}; do
    set -- ${CFG//,/ }
    timeout -k 10 300 python bench.py --objects $1 --chains $2 --iters $3 --steps $4 --warmup 1 \
        --no-cpu-baseline > $OUT/${V}_n$1.json 2> $OUT/${V}_n$1.err || { tail -5 $OUT/${V}_n$1.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/${V}_n$1.json').read().strip().splitlines()[-1]); c=d['config']; print('$V N=$1 value=%.4g ms/launch=%.2f resident=%s' % (d['value'], d['kernel_ms_per_launch'], c.get('resident_chains_per_cu')))"
  done
done
