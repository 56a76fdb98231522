#!/bin/bash
# On the GPU box: per-phase instruction counts of the step kernel from the MH_DOUBLE probe
# builds (tools/build_ablate.sh dbl1 dbl4 ...). Each probe runs one phase twice with identical
# results, so (probe - base) counters = that phase's cost. One PMC pass per variant.
#   tools/phase_cost_box.sh <tag> <variant>...
set -o pipefail
TAG=${1:-phase}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
CNT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for M in 0 "$@"; do
  if [ "$M" = 0 ]; then LIB=metropolis-hastings-gpgpu_amd/libmhgpu.so; else LIB=abvar/libmhgpu_$M.so; fi
  MH_LIB=$LIB timeout -k 10 300 rocprofv3 --pmc $CNT -d "$OUT/pmc_$M" -o pmc --output-format csv \
      -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_$M.log" 2>&1 || { echo "variant $M failed"; tail -5 "$OUT/pmc_$M.log"; exit 1; }
done
echo "phase costs $TAG done"
