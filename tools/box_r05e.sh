#!/bin/bash
# Round 5: per-phase stamps of the speculative kernel v3, the speculative / default choice at
# larger chain counts, and config 5 against round 4's library (the replay's value loads).
set -o pipefail
TAG=${1:-r05e}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
MH_SPEC=1 timeout -k 10 120 python tools/stamps.py 8 1024 2000 > $OUT/stamps_spec_n8.txt 2>&1 || { tail -5 $OUT/stamps_spec_n8.txt; exit 1; }
cat $OUT/stamps_spec_n8.txt
for CH in 2560 3072 4096 8192; do
  for SPEC in 1 0; do
    MH_SPEC=$SPEC timeout -k 10 120 python bench.py --objects 8 --chains $CH --iters 2000 --steps 4 \
        --warmup 1 --no-cpu-baseline --e2e-iters 0 > $OUT/spec${SPEC}_$CH.json 2> $OUT/spec${SPEC}_$CH.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/spec${SPEC}_$CH.json').read().strip().splitlines()[-1]); print('MH_SPEC=$SPEC N=8 $CH chains value=%.4g ms/launch=%.3f kernel=%s resident/CU=%s' % (d['value'], d['kernel_ms_per_launch'], d['config'].get('step_kernel'), d['config'].get('resident_chains_per_cu')))"
  done
done
MH_AB_REPS=3 MH_AB_CFGS="256,32768,1000,2" bash tools/box_abn.sh $TAG/ab main r04 || exit 1
