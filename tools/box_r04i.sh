#!/bin/bash
# Round 4: speculative kernel timing (MH_SPEC=1) against the few-chains kernel at config 2, and
# per-phase cycles with the scan split into lane parse / walk / group records.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r04i}; mkdir -p $OUT
MH_SPEC=1 timeout -k 10 120 python -u tools/stamps.py 8 1024 2000 > $OUT/stamps_spec.txt 2>&1; rc=$?; cat $OUT/stamps_spec.txt; [ $rc = 0 ] || exit 1
for rep in 1 2; do
  for SP in 0 1; do
    MH_SPEC=$SP timeout -k 10 240 python bench.py --objects 8 --chains 1024 --iters 2000 --steps 4 \
        --warmup 1 --no-cpu-baseline --e2e-iters 0 > $OUT/b_${SP}_${rep}.json 2> $OUT/b_${SP}_${rep}.err || { tail -5 $OUT/b_${SP}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/b_${SP}_${rep}.json').read().strip().splitlines()[-1]); print('MH_SPEC=$SP rep $rep value=%.4g ms/launch=%.3f mean=%.10g acc=%d kernel=%s' % (d['value'], d['kernel_ms_per_launch'], d['mean_final_cost'], d['accepted'], d['config'].get('step_kernel')))"
  done
done
