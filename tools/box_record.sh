#!/bin/bash
# On the GPU box: a round's record of the three measured configs. For each: kernel trace + the
# PMC passes (tools/profile_box.sh), the step kernel's record (tools/pmc_summary.py --json) put
# where bench.py reads it (profiles/pmc_step_kernel_n<N>.json, so the bench line that follows
# reports it as current), then the bench line. Outputs under gpurun_out/<tag>/; copy the records,
# summaries, kernel stats and bench lines into profiles/.
#   tools/box_record.sh <tag>
set -o pipefail
TAG=${1:-record}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
# N, step-kernel name substring, chains, profile args, bench args
one() {
  local N=$1 K=$2 CH=$3 PARGS=$4 BARGS=$5
  bash tools/profile_box.sh $TAG/n$N $PARGS || return 1
  python tools/pmc_summary.py $OUT/n$N --kernel "$K" --chains $CH \
      --json $OUT/pmc_step_kernel_n$N.json > $OUT/pmc_n$N.txt || return 1
  cp $OUT/pmc_step_kernel_n$N.json profiles/pmc_step_kernel_n$N.json
  head -12 $OUT/pmc_n$N.txt
  timeout -k 10 400 python bench.py $BARGS > $OUT/bench_n$N.json 2> $OUT/bench_n$N.err \
      || { tail -5 $OUT/bench_n$N.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('N=%s value=%.4g ms/launch=%.3f frac=%.4f pmc=%s valu/step=%s' % (sys.argv[2], d['value'], d['kernel_ms_per_launch'], r['frac'], r.get('pmc_status'), r.get('executed_valu_wave_insts_per_chain_step')))" $OUT/bench_n$N.json $N
}
one 64 "mh_kernel<64, 1, 1>" 65536 "--steps 3 --warmup 1 --iters 1000 --no-cpu-baseline --e2e-iters 0" \
    "--steps 20 --warmup 5" || exit 1
one 256 "mh_delta_kernel" 32768 \
    "--objects 256 --chains 32768 --steps 3 --warmup 1 --iters 1000 --no-cpu-baseline --e2e-iters 0" \
    "--objects 256 --chains 32768 --iters 1000 --steps 8 --warmup 2 --no-cpu-baseline" || exit 1
one 8 "mh_spec_kernel" 1024 \
    "--objects 8 --chains 1024 --steps 3 --warmup 1 --iters 1000 --no-cpu-baseline --e2e-iters 0" \
    "--objects 8 --chains 1024 --iters 2000 --steps 4 --warmup 1 --no-cpu-baseline" || exit 1
echo "box_record.sh $TAG: done"
