#!/bin/bash
# On the GPU box: the counting build's bound decisions and list lengths (tools/stamps.py on
# abvar/libmhgpu_counts.so) for configs 5 and 3.   tools/box_counts.sh <tag>
set -o pipefail
TAG=${1:-counts}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
export MH_LIB=abvar/libmhgpu_counts.so
for CFG in "64 65536 1000" "256 32768 1000"; do
  set -- $CFG
  timeout -k 10 150 python tools/stamps.py $1 $2 $3 > $OUT/counts_n$1.txt 2>&1 || { cat $OUT/counts_n$1.txt; exit 1; }
  cat $OUT/counts_n$1.txt
done
