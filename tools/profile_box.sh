#!/bin/bash
# Runs on the GPU box (via gpurun) from the repo root. Writes raw rocprofv3 output under
# gpurun_out/<tag>/; copy the summaries worth keeping into profiles/.
#   tools/profile_box.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-prof}; shift
ARGS=${@:---steps 5 --warmup 1 --no-cpu-baseline}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
# the source hash of the library these passes profile (bench.py trusts a PMC record only for it)
LIB=${MH_LIB:-metropolis-hastings-gpgpu_amd/libmhgpu.so}
if [ -f "$LIB.srchash" ]; then cp "$LIB.srchash" "$OUT/srchash"; else echo "(no record)" > "$OUT/srchash"; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv \
    -- python3 bench.py $ARGS > "$OUT/kt.log" 2>&1 || { echo "kernel-trace pass failed"; exit 1; }
for PASS in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
    "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_CVT" \
    "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"; do
  NAME=$(echo "$PASS" | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $PASS -d "$OUT/pmc_$NAME" -o pmc --output-format csv \
      -- python3 bench.py $ARGS > "$OUT/pmc_$NAME.log" 2>&1 || { echo "pmc pass $NAME failed"; tail -5 "$OUT/pmc_$NAME.log"; exit 1; }
done
echo "profile $TAG done"
