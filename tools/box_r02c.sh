#!/bin/bash
# On the GPU box: GPU tests, short benches of configs 3 / 5 / 2, and per-phase stamps of the
# three step kernels (ablate/libmhgpu_stamps.so).   tools/box_r02c.sh <tag> [nopytest]
set -o pipefail
TAG=${1:-r02c}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
rc=0
if [ "$2" != "nopytest" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
      -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; rc=$?
  tail -15 $OUT/pytest_gpu.log
  [ $rc -le 1 ] || { echo "pytest ended with $rc: stopping"; exit $rc; }
fi
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 \
    > $OUT/bench_n64.json 2> $OUT/bench_n64.err || { tail -5 $OUT/bench_n64.err; exit 1; }
tail -1 $OUT/bench_n64.json | cut -c1-300
timeout -k 10 300 python bench.py --no-cpu-baseline --objects 256 --chains 32768 --iters 1000 \
    --steps 3 --warmup 1 > $OUT/bench_n256.json 2> $OUT/bench_n256.err || { tail -5 $OUT/bench_n256.err; exit 1; }
tail -1 $OUT/bench_n256.json | cut -c1-300
timeout -k 10 120 python bench.py --no-cpu-baseline --objects 8 --chains 1024 --iters 1000 \
    --steps 5 --warmup 1 > $OUT/bench_n8.json 2> $OUT/bench_n8.err || { tail -5 $OUT/bench_n8.err; exit 1; }
tail -1 $OUT/bench_n8.json | cut -c1-300
if [ -f ablate/libmhgpu_stamps.so ]; then
  export MH_LIB=ablate/libmhgpu_stamps.so
  timeout -k 10 120 python tools/stamps.py 64 65536 300 > $OUT/stamps_n64.txt 2>&1 || { cat $OUT/stamps_n64.txt; exit 1; }
  cat $OUT/stamps_n64.txt
  timeout -k 10 120 python tools/stamps.py 256 32768 200 > $OUT/stamps_n256.txt 2>&1 || { cat $OUT/stamps_n256.txt; exit 1; }
  cat $OUT/stamps_n256.txt
  timeout -k 10 120 python tools/stamps.py 8 1024 3000 > $OUT/stamps_n8.txt 2>&1 || { cat $OUT/stamps_n8.txt; exit 1; }
  cat $OUT/stamps_n8.txt
fi
exit $rc
