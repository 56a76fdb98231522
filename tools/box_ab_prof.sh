#!/bin/bash
# On the GPU box: tools/box_ab.sh (GPU suite + variant A/B at config 3), then the config-3
# kernel-trace and PMC passes of the product library.   tools/box_ab_prof.sh <tag> <variant>...
set -o pipefail
TAG=${1:-abp}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/box_ab.sh "$@" || exit 1
OUT=gpurun_out/$TAG
bash tools/profile_box.sh $TAG/n64 --steps 3 --warmup 1 --iters 1000 --no-cpu-baseline || exit 1
python tools/pmc_summary.py $OUT/n64 --kernel "mh_kernel<64, 1, 1>" --chains 65536 \
    --json $OUT/pmc_step_kernel_n64.json > $OUT/pmc_n64.txt || exit 1
grep -E 'duration_ns|hbm_|valu_issue_util |valu_insts_per_wave' $OUT/pmc_n64.txt
