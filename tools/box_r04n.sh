#!/bin/bash
# Round 4: the shared math with fused multiply-adds (atan, exp, sin/cos kernels): device ==
# oracle on every probe (exhaustive and sampled), parity of the step kernels, A/B against HEAD.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r04n}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_math.py -m gpu -x -v --timeout 600 --timeout-method thread \
    -p no:cacheprovider -W always::UserWarning > $OUT/pytest_math.log 2>&1 || { tail -40 $OUT/pytest_math.log; exit 1; }
grep -E "passed|failed" $OUT/pytest_math.log | tail -1
grep -E "MathReport" $OUT/pytest_math.log | sed 's/.*MathReport: //' | sort -u | awk '{print $3, $4, $NF}' | tr '\n' ';'; echo
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spec.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_parity.log 2>&1 || { tail -40 $OUT/pytest_parity.log; exit 1; }
tail -1 $OUT/pytest_parity.log
MH_AB_REPS=2 MH_AB_CFGS="8,1024,2000,4 256,32768,1000,1 64,65536,1000,3" bash tools/box_abn.sh ${1:-r04n}/ab prev ocml2 main
