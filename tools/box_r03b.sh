#!/bin/bash
# On the GPU box: the counting build's bound decisions for configs 3 and 5 (round 2's faulted
# leg, re-run on the inlined build), then per-phase stamps of configs 3, 5 and 2.
set -o pipefail
TAG=${1:-r03b}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/box_counts.sh $TAG/counts && bash tools/box_stamps.sh $TAG/stamps
