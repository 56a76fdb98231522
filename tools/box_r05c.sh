#!/bin/bash
# Round 5: the whole GPU suite at the current sources, then the speculative / few-chains choice
# for N = 8 across chain counts (the cutoff in choose_geometry).
set -o pipefail
TAG=${1:-r05c}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest_gpu.log | tail -15; [ $rc -eq 0 ] || exit $rc
for CH in 1280 1536 1792; do
  for SPEC in 1 0; do
    MH_SPEC=$SPEC timeout -k 10 120 python bench.py --objects 8 --chains $CH --iters 2000 --steps 4 \
        --warmup 1 --no-cpu-baseline --e2e-iters 0 > $OUT/spec${SPEC}_$CH.json 2> $OUT/spec${SPEC}_$CH.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/spec${SPEC}_$CH.json').read().strip().splitlines()[-1]); print('MH_SPEC=$SPEC N=8 $CH chains value=%.4g ms/launch=%.3f kernel=%s' % (d['value'], d['kernel_ms_per_launch'], d['config'].get('step_kernel')))"
  done
done
if [ -f ablate/libmhgpu_stamps.so ]; then
  MH_SPEC=1 timeout -k 10 120 python tools/stamps.py 8 1024 2000 > $OUT/stamps_spec_n8.txt 2>&1 || { tail -5 $OUT/stamps_spec_n8.txt; exit 1; }
  cat $OUT/stamps_spec_n8.txt
  timeout -k 10 180 python tools/stamps.py 64 65536 1000 > $OUT/stamps_n64.txt 2>&1 || { tail -5 $OUT/stamps_n64.txt; exit 1; }
  cat $OUT/stamps_n64.txt
  timeout -k 10 180 python tools/stamps.py 256 32768 1000 > $OUT/stamps_n256.txt 2>&1 || { tail -5 $OUT/stamps_n256.txt; exit 1; }
  cat $OUT/stamps_n256.txt
fi
