#!/bin/bash
# On the GPU box: the round's measurement record. The GPU suite; the bench line of each config
# with its CPU baseline (config 3 also with the end-to-end KernelWrapper leg); then kernel-trace
# and PMC passes of each config's step kernel (tools/profile_box.sh), summarised by
# tools/pmc_summary.py into the records bench.py reads.   tools/box_measure.sh <tag>
set -o pipefail
TAG=${1:-measure}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
# (config 3: the driver's shape; config 5: 10k steps; config 2: 10k steps)
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_n64.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
timeout -k 10 300 python bench.py --objects 256 --chains 32768 --iters 1000 --steps 8 --warmup 2 --e2e-iters 1000 > $OUT/bench_n256.json 2>> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
timeout -k 10 300 python bench.py --objects 8 --chains 1024 --iters 2000 --steps 4 --warmup 1 --e2e-iters 2000 > $OUT/bench_n8.json 2>> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
for f in n64 n256 n8; do python -c "import json; d=json.loads(open('$OUT/bench_$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['kernel_ms_per_launch'], d['mean_final_cost'], d['cpu_baseline']['value'], d['e2e_chain_steps_per_s'])"; done
bash tools/profile_box.sh $TAG/n64 --steps 3 --warmup 1 --iters 1000 --no-cpu-baseline --e2e-iters 0 || exit 1
python tools/pmc_summary.py $OUT/n64 --kernel "mh_kernel<64, 1, 1>" --chains 65536 \
    --json $OUT/pmc_step_kernel_n64.json --profile profiles/${TAG}_pmc_step_kernel_n64.txt > $OUT/pmc_n64.txt || exit 1
bash tools/profile_box.sh $TAG/n256 --objects 256 --chains 32768 --steps 3 --warmup 1 --iters 1000 --no-cpu-baseline --e2e-iters 0 || exit 1
python tools/pmc_summary.py $OUT/n256 --kernel "mh_delta_kernel" --chains 32768 \
    --json $OUT/pmc_step_kernel_n256.json --profile profiles/${TAG}_pmc_step_kernel_n256.txt > $OUT/pmc_n256.txt || exit 1
bash tools/profile_box.sh $TAG/n8 --objects 8 --chains 1024 --steps 3 --warmup 1 --iters 1000 --no-cpu-baseline --e2e-iters 0 || exit 1
python tools/pmc_summary.py $OUT/n8 --kernel "mh_spec_kernel" --chains 1024 \
    --json $OUT/pmc_step_kernel_n8.json --profile profiles/${TAG}_pmc_step_kernel_n8.txt > $OUT/pmc_n8.txt || exit 1
cat $OUT/pmc_n64.txt $OUT/pmc_n256.txt $OUT/pmc_n8.txt | grep -E "hbm_bytes|valu_issue|insts_per_wave|duration|Scratch|wait_inst"
