#!/bin/bash
# On the GPU box: per-phase cycle stamps (abvar/libmhgpu_stamps.so, tools/build_ablate.sh
# stamps) of config 3, config 5 and config 2.   tools/box_stamps.sh <tag>
set -o pipefail
TAG=${1:-stamps}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
export MH_LIB=abvar/libmhgpu_stamps.so
timeout -k 10 120 python tools/stamps.py 64 65536 1000 > $OUT/stamps_n64.txt 2>&1 || { cat $OUT/stamps_n64.txt; exit 1; }
cat $OUT/stamps_n64.txt
timeout -k 10 120 python tools/stamps.py 256 32768 300 > $OUT/stamps_n256.txt 2>&1 || { cat $OUT/stamps_n256.txt; exit 1; }
cat $OUT/stamps_n256.txt
timeout -k 10 120 python tools/stamps.py 8 1024 3000 > $OUT/stamps_n8.txt 2>&1 || { cat $OUT/stamps_n8.txt; exit 1; }
cat $OUT/stamps_n8.txt
