#!/bin/bash
# On the GPU box: canary, the incremental-kernel GPU tests, the config-5 bench and its stamps.
#   tools/box_n256.sh <tag>
set -o pipefail
TAG=${1:-n256}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 120 python -u tools/canary.py || { echo "canary failed: stopping"; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread \
    -p no:cacheprovider -k "incremental or config5 or index_n or overflow" > $OUT/pytest_gpu.log 2>&1 \
    || { tail -20 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --objects 256 --chains 32768 --iters 1000 --steps 3 --warmup 1 \
    --no-cpu-baseline > $OUT/bench_n256.json 2> $OUT/bench_n256.err || { tail -5 $OUT/bench_n256.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_n256.json').read().strip().splitlines()[-1]); print('N=256 value=%.4g ms/launch=%.2f mean=%.6g resident=%s' % (d['value'], d['kernel_ms_per_launch'], d['mean_final_cost'], d['config']['resident_chains_per_cu']))"
MH_LIB=abvar/libmhgpu_stamps.so timeout -k 10 120 python tools/stamps.py 256 32768 300 > $OUT/stamps_n256.txt 2>&1 || { cat $OUT/stamps_n256.txt; exit 1; }
cat $OUT/stamps_n256.txt
