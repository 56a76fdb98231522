#!/bin/bash
# On the GPU box: bench each ablation variant built by tools/build_ablate.sh.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=${1:-32}; shift
for M in 0 "$@"; do
  if [ "$M" = 0 ]; then LIB=metropolis-hastings-gpgpu_amd/libmhgpu.so; else LIB=abvar/libmhgpu_$M.so; fi
  MH_LANES=$L MH_LIB=$LIB timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abl_L${L}_$M.log 2>&1 || { echo "variant $M failed"; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/abl_L${L}_$M.log').read().strip().splitlines()[-1]); print('L=$L ablate=$M kernel_ms=%.1f value=%.4g' % (d['kernel_ms_per_step'], d['value']))"
done
