#!/bin/bash
# On the GPU box: the GPU test suite, then an A/B of library variants at config 3 (timing only,
# alternating so drift hits both).   tools/box_ab.sh <tag> <variant>...  ("main" = the product)
set -o pipefail
TAG=${1:-ab}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest_gpu.log
bash tools/box_variants.sh $TAG "$@"
