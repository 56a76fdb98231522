#!/bin/bash
# On the GPU box: GPU tests, per-phase instruction costs (MH_DOUBLE probes) and stamps of the
# config-3 step kernel, config 2 with the default (widened) geometry.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r02b; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -15 $OUT/pytest_gpu.log
[ $rc -le 1 ] || { echo "pytest ended with $rc: stopping"; exit $rc; }
timeout -k 10 120 python bench.py --objects 8 --chains 1024 --iters 1000 --steps 5 --warmup 1 \
    --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err || exit 1
tail -1 $OUT/c2.json | cut -c1-400
bash tools/phase_cost_box.sh r02b/phase dbl1 dbl64 dbl4 dbl8 dbl16 dbl32 || exit 1
python tools/phase_cost.py $OUT/phase
MH_LIB=ablate/libmhgpu_stamps.so timeout -k 10 120 python tools/stamps.py 64 65536 300 > $OUT/stamps64.txt 2>&1 || exit 1
cat $OUT/stamps64.txt
exit $rc
