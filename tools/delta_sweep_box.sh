#!/bin/bash
# On the GPU box: bench the incremental step kernel at each lanes-per-chain shape against the
# full-evaluation step kernel.   tools/delta_sweep_box.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-sweep}; shift
ARGS=${@:---steps 3 --warmup 1 --no-cpu-baseline}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
for V in "0 0" "1 8" "1 16" "1 32"; do
  set -- $V
  MH_DELTA=$1 MH_DELTA_LANES=$2 timeout -k 10 300 python bench.py $ARGS > gpurun_out/$TAG/d$1_L$2.json 2> gpurun_out/$TAG/d$1_L$2.err || { echo "variant $V failed"; tail -3 gpurun_out/$TAG/d$1_L$2.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/$TAG/d$1_L$2.json').read().strip().splitlines()[-1]); print('delta=$1 L=$2 value=%.4g kernel_ms=%.1f lanes=%s cpw=%s mean=%.6g' % (d['value'], d['kernel_ms_per_step'], d['config']['lanes_per_chain'], d['config']['chains_per_workgroup'], d['mean_final_cost']))"
done
