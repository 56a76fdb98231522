#!/bin/bash
# Round 5 measurement record, on the GPU box (the full GPU suite and smoke() first). PMC and kernel-trace passes of each config's step
# kernel first (tools/profile_box.sh), their records written into this box's profiles/ so the
# bench lines that follow read them as current; then the bench line of each config with its CPU
# baseline and end-to-end KernelWrapper leg; finally the default bench line (the driver's).
#   tools/box_r05m.sh <tag>
set -o pipefail
TAG=${1:-r05s}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log; cp $OUT/pytest_gpu.log profiles/${TAG}_pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log; cp $OUT/smoke.log profiles/${TAG}_smoke.txt
prof() {  # name kernel chains bench-args...
  local NAME=$1 KERN=$2 CH=$3; shift 3
  bash tools/profile_box.sh $TAG/$NAME "$@" || return 1
  python tools/pmc_summary.py $OUT/$NAME --kernel "$KERN" --chains $CH \
      --json $OUT/pmc_step_kernel_$NAME.json --profile profiles/${TAG}_pmc_step_kernel_$NAME.txt \
      > $OUT/pmc_$NAME.txt || return 1
  cp $OUT/pmc_step_kernel_$NAME.json profiles/pmc_step_kernel_$NAME.json
  cp $OUT/pmc_$NAME.txt profiles/${TAG}_pmc_step_kernel_$NAME.txt
  cp $OUT/$NAME/kt/kt_kernel_stats.csv profiles/${TAG}_kernel_stats_$NAME.csv 2>/dev/null || \
      find $OUT/$NAME/kt -name "*kernel_stats.csv" -exec cp {} profiles/${TAG}_kernel_stats_$NAME.csv \;
}
prof n64 "mh_kernel<64, 1, 1>" 65536 --steps 3 --warmup 1 --iters 1000 --no-cpu-baseline --e2e-iters 0 || exit 1
prof n256 "mh_delta_kernel" 32768 --objects 256 --chains 32768 --steps 3 --warmup 1 --iters 1000 --no-cpu-baseline --e2e-iters 0 || exit 1
prof n8 "mh_spec_kernel" 1024 --objects 8 --chains 1024 --steps 3 --warmup 1 --iters 1000 --no-cpu-baseline --e2e-iters 0 || exit 1
grep -hE "hbm_bytes|valu_issue|insts_per_wave|duration|wait_inst" $OUT/pmc_n64.txt $OUT/pmc_n256.txt $OUT/pmc_n8.txt
timeout -k 10 300 python bench.py --objects 256 --chains 32768 --iters 1000 --steps 8 --warmup 2 --e2e-iters 1000 > $OUT/bench_n256.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
timeout -k 10 300 python bench.py --objects 8 --chains 1024 --iters 2000 --steps 4 --warmup 1 --e2e-iters 2000 > $OUT/bench_n8.json 2>> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_n64.json 2>> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
for f in n64 n256 n8; do python -c "import json; d=json.loads(open('$OUT/bench_$f.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$f value %.4g ms/launch %.3f frac %.4f traffic %s pmc %s cpu %.3g e2e %s mean %.9g' % (d['value'], d['kernel_ms_per_launch'], r['frac'], r['traffic'], r['pmc_status'], d['cpu_baseline']['value'], d['e2e_chain_steps_per_s'], d['mean_final_cost']))"; done
cp $OUT/bench_n64.json profiles/${TAG}_bench_n64.json; cp $OUT/bench_n256.json profiles/${TAG}_bench_n256.json; cp $OUT/bench_n8.json profiles/${TAG}_bench_n8.json
mkdir -p $OUT/profiles && cp profiles/pmc_step_kernel_n*.json profiles/${TAG}_* $OUT/profiles/
