#!/bin/bash
# On the GPU box: GPU tests (optionally a -k filter), then the config-3 bench (and config 5 /
# config 2 lines).   tools/box_quick.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-quick}; K=${2:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 120 python -u tools/canary.py || { echo "canary failed: stopping"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 170 --timeout-method thread \
    -p no:cacheprovider "${KARG[@]}" > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -6 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest ended with $rc: stopping"; grep -E "Error|assert|FAILED" $OUT/pytest_gpu.log | head -20; exit $rc; }
for CFG in "64 65536 4000 5" "256 32768 1000 5" "8 1024 1000 5"; do
  set -- $CFG
  timeout -k 10 300 python bench.py --objects $1 --chains $2 --iters $3 --steps $4 --warmup 1 \
      --no-cpu-baseline > $OUT/bench_n$1.json 2> $OUT/bench_n$1.err || { tail -5 $OUT/bench_n$1.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_n$1.json').read().strip().splitlines()[-1]); print('N=$1 value=%.4g ms/launch=%.2f mean=%.6g frac=%.4f' % (d['value'], d['kernel_ms_per_launch'], d['mean_final_cost'], d['roofline']['frac']))"
done
