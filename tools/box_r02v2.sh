#!/bin/bash
# On the GPU box: profiles of the current build -- the default bench line (cpu_baseline
# included), kernel-trace + PMC passes of configs 3 and 5 (tools/box_prof.sh), and per-phase
# stamps with the list / bound counts (ablate/libmhgpu_counts.so) of configs 3, 5 and 2.
#   tools/box_r02v2.sh <tag>
set -o pipefail
TAG=${1:-r02_v2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/box_prof.sh $TAG || exit 1
export MH_LIB=ablate/libmhgpu_counts.so
for CFG in "64 65536 300" "256 32768 200" "8 1024 3000"; do
  set -- $CFG
  timeout -k 10 120 python tools/stamps.py $1 $2 $3 > $OUT/stamps_n$1.txt 2>&1 || { cat $OUT/stamps_n$1.txt; exit 1; }
  cat $OUT/stamps_n$1.txt
done
