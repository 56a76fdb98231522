#!/bin/bash
# On the GPU box: profiles of the current build -- the default bench line (cpu_baseline
# included), kernel-trace + PMC passes of configs 3 and 5 (tools/box_prof.sh), and per-phase
# stamps (ablate/libmhgpu_stamps.so) of configs 5, 3 and 2.   tools/box_r02v3.sh <tag>
set -o pipefail
TAG=${1:-r02_v3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/box_prof.sh $TAG || exit 1
export MH_LIB=ablate/libmhgpu_stamps.so
for CFG in "256 32768 300" "64 65536 300" "8 1024 3000"; do
  set -- $CFG
  timeout -k 10 120 python tools/stamps.py $1 $2 $3 > $OUT/stamps_n$1.txt 2>&1 || { cat $OUT/stamps_n$1.txt; exit 1; }
  cat $OUT/stamps_n$1.txt
done
