#!/bin/bash
# On the GPU box: the default bench line (cpu_baseline included), then kernel-trace + PMC passes
# of config 3 and config 5 (tools/profile_box.sh), summarised by tools/pmc_summary.py.
#   tools/box_prof.sh <tag>
set -o pipefail
TAG=${1:-prof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 240 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err \
    || { tail -5 $OUT/bench_default.err; exit 1; }
tail -1 $OUT/bench_default.json | cut -c1-600
bash tools/profile_box.sh $TAG/n64 --steps 3 --warmup 1 --iters 1000 --no-cpu-baseline || exit 1
python tools/pmc_summary.py $OUT/n64 --kernel "mh_kernel<64, 1, 1>" --chains 65536 \
    --json $OUT/pmc_step_kernel_n64.json > $OUT/pmc_n64.txt || exit 1
cat $OUT/pmc_n64.txt
bash tools/profile_box.sh $TAG/n256 --objects 256 --chains 32768 --steps 3 --warmup 1 \
    --iters 1000 --no-cpu-baseline || exit 1
python tools/pmc_summary.py $OUT/n256 --kernel "mh_delta_kernel" --chains 32768 \
    --json $OUT/pmc_step_kernel_n256.json > $OUT/pmc_n256.txt || exit 1
cat $OUT/pmc_n256.txt
