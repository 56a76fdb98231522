#!/bin/bash
# On the GPU box: A/B of library variants (abvar/libmhgpu_<v>.so; "main" = the product) over
# several configs, alternated $MH_AB_REPS times so drift hits every variant. Prints value and
# mean final cost per run (equal means across variants: the same trajectories).
#   MH_AB_CFGS="8,1024,2000,4 64,65536,1000,3" tools/box_abn.sh <tag> <variant>...
# (a variant: a library name, "main" = the product, optionally with environment settings after
# colons, e.g. main:MH_SPEC_H=1)
set -o pipefail
TAG=${1:-abn}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in $(seq 1 ${MH_AB_REPS:-2}); do
  for CFG in ${MH_AB_CFGS:-8,1024,2000,4 64,65536,1000,3}; do
    set -- ${CFG//,/ } "${@}"
    N=$1; CH=$2; IT=$3; ST=$4; shift 4
    for V in "$@"; do
      # a variant is a library name ("main" = the product) with optional environment settings
      # after colons: main:MH_SPEC_H=1:MH_SPEC=1
      LV=${V%%:*}; ENVS=""; [ "$LV" != "$V" ] && ENVS=$(echo "${V#*:}" | tr ':' ' ')
      if [ "$LV" = main ]; then LIB=metropolis-hastings-gpgpu_amd/libmhgpu.so; else LIB=abvar/libmhgpu_$LV.so; fi
      F=$OUT/$(echo "$V" | tr ':=' '__')_n${N}_$rep
      env $ENVS MH_LIB=$LIB timeout -k 10 240 python bench.py --objects $N --chains $CH --iters $IT --steps $ST \
          --warmup 1 --no-cpu-baseline --e2e-iters 0 > $F.json 2> $F.err || { tail -5 $F.err; exit 1; }
      python -c "import json; d=json.loads(open('$F.json').read().strip().splitlines()[-1]); print('$V N=$N rep $rep value=%.4g ms/launch=%.3f mean=%.10g acc=%d' % (d['value'], d['kernel_ms_per_launch'], d['mean_final_cost'], d['accepted']))"
    done
  done
done
