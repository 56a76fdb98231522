#!/bin/bash
# Round 4: config 5 residency. Incremental-kernel parity after the LDS cut (no cached object
# boxes, Clearance list capacity 2 per object), then an A/B at config 5: HEAD~ (8 chains per
# CU), the product (LDS for 12, VGPRs for 8) and dw12 (the kernel capped at 168 VGPRs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r04j}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider -W always::UserWarning -k "incremental or config5 or overflow" \
    > $OUT/pytest_delta.log 2>&1 || { tail -40 $OUT/pytest_delta.log; exit 1; }
grep -E "passed|failed" $OUT/pytest_delta.log | tail -2
for rep in 1 2; do
  for V in head main dw12; do
    if [ "$V" = main ]; then LIB=metropolis-hastings-gpgpu_amd/libmhgpu.so; else LIB=ablate/libmhgpu_$V.so; fi
    F=$OUT/${V}_$rep
    MH_LIB=$LIB timeout -k 10 240 python bench.py --objects 256 --chains 32768 --iters 1000 --steps 1 \
        --warmup 1 --no-cpu-baseline --e2e-iters 0 > $F.json 2> $F.err || { tail -5 $F.err; exit 1; }
    python -c "import json; d=json.loads(open('$F.json').read().strip().splitlines()[-1]); print('$V rep $rep value=%.4g ms/launch=%.3f mean=%.10g acc=%d resident=%s' % (d['value'], d['kernel_ms_per_launch'], d['mean_final_cost'], d['accepted'], d['config'].get('resident_chains_per_cu')))"
  done
done
MH_SPEC=1 timeout -k 10 120 python -u tools/stamps.py 8 1024 2000 > $OUT/stamps_spec.txt 2>&1; rc=$?; cat $OUT/stamps_spec.txt; [ $rc = 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_spec.log 2>&1 || { tail -40 $OUT/pytest_spec.log; exit 1; }
tail -1 $OUT/pytest_spec.log
for rep in 1 2; do
  for SP in 0 1; do
    MH_SPEC=$SP timeout -k 10 240 python bench.py --objects 8 --chains 1024 --iters 2000 --steps 4 \
        --warmup 1 --no-cpu-baseline --e2e-iters 0 > $OUT/b_${SP}_$rep.json 2> $OUT/b_${SP}_$rep.err || { tail -5 $OUT/b_${SP}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/b_${SP}_$rep.json').read().strip().splitlines()[-1]); print('MH_SPEC=$SP rep $rep value=%.4g ms/launch=%.3f mean=%.10g acc=%d' % (d['value'], d['kernel_ms_per_launch'], d['mean_final_cost'], d['accepted']))"
  done
done
