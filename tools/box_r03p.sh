#!/bin/bash
# Round 3 probes: per-phase LDS bank conflicts / instruction counts (MH_DOUBLE probe builds) and
# the two-chains-per-wavefront A/B at config 3 (MH_LANES=32).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03p
mkdir -p $OUT
timeout -k 10 600 bash tools/phase_cost_box.sh r03p dbl1 dbl64 dbl128 dbl256 || exit 1
python3 tools/phase_cost.py gpurun_out/r03p > $OUT/phase_costs.txt || exit 1
cat $OUT/phase_costs.txt
MH_LANES=32 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --e2e-iters 0 > $OUT/bench_l32.json 2> $OUT/bench_l32.err || exit 1
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --e2e-iters 0 > $OUT/bench_l64.json 2> $OUT/bench_l64.err || exit 1
cat $OUT/bench_l32.json $OUT/bench_l64.json
