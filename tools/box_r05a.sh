#!/bin/bash
# Round 5, first box run: the out-of-line build against the product (tools/box_fault4.sh: costs
# bit-identical at 256 / 4,096 / 65,536 chains), then an A/B of the product (type punning
# removed) against round 4's library (ablate/libmhgpu_r04.so) on configs 2, 3 and 5.
set -o pipefail
TAG=${1:-r05a}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
bash tools/box_fault4.sh $TAG/fault || exit 1
MH_AB_REPS=3 MH_AB_CFGS="8,1024,2000,4 64,65536,1000,3 256,32768,1000,2" \
    bash tools/box_abn.sh $TAG/ab main r04
