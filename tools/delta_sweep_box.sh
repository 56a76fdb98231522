#!/bin/bash
# On the GPU box: bench the incremental step kernel (at the chooser's workgroup size and at
# pinned sizes) against the full-evaluation step kernel.   tools/delta_sweep_box.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-sweep}; shift
ARGS=${@:---steps 3 --warmup 1 --no-cpu-baseline}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$TAG
for V in "0 0" "1 0" "1 4" "1 8"; do
  set -- $V
  if [ "$2" = 0 ]; then unset MH_DELTA_WAVES; else export MH_DELTA_WAVES=$2; fi
  MH_DELTA=$1 timeout -k 10 300 python bench.py $ARGS > gpurun_out/$TAG/d$1_w$2.json 2> gpurun_out/$TAG/d$1_w$2.err || { echo "variant $V failed"; tail -3 gpurun_out/$TAG/d$1_w$2.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/$TAG/d$1_w$2.json').read().strip().splitlines()[-1]); c=d['config']; print('delta=$1 waves=$2 value=%.4g kernel_ms=%.1f cpw=%s resident=%s mean=%.6g' % (d['value'], d['kernel_ms_per_step'], c['chains_per_workgroup'], c.get('resident_chains_per_cu'), d['mean_final_cost']))"
done
