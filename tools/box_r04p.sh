#!/bin/bash
# Round 4: the speculative kernel split over two wavefronts per chain: parity, stamps, A/B against
# the one-wavefront version (HEAD).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r04p}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider -W always::UserWarning > $OUT/pytest_spec.log 2>&1 || { tail -40 $OUT/pytest_spec.log; exit 1; }
grep -E "passed|failed" $OUT/pytest_spec.log | tail -1
MH_SPEC=1 timeout -k 10 120 python -u tools/stamps.py 8 1024 2000 > $OUT/stamps_spec.txt 2>&1; rc=$?; cat $OUT/stamps_spec.txt; [ $rc = 0 ] || exit 1
MH_AB_REPS=2 MH_AB_CFGS="8,1024,2000,4" bash tools/box_abn.sh ${1:-r04p}/ab split main
