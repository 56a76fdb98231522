#!/bin/bash
# LDS bank conflicts of config 3's step kernel per phase: the product against MH_ABLATE builds
# that compile one phase out (1 symmetry rows, 2 per-object atan2/cos, 8 SurfaceArea/Clearance
# pairs, 32 Box-Muller). Timing-only builds: their results are wrong by construction.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-ldsconf}; mkdir -p $OUT
ARGS="--steps 1 --warmup 1 --iters 1000 --no-cpu-baseline --e2e-iters 0"
for V in main 1 2 8 32; do
  if [ "$V" = main ]; then LIB=metropolis-hastings-gpgpu_amd/libmhgpu.so; else LIB=abvar/libmhgpu_$V.so; fi
  MH_LIB=$LIB timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU \
      -d $OUT/pmc_$V -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_$V.log 2>&1 || { tail -5 $OUT/pmc_$V.log; exit 1; }
  python3 - "$OUT/pmc_$V" "$V" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection*.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "mh_kernel<64, 1, 1>" in row.get("Kernel_Name", ""):
            agg[row["Counter_Name"]] += float(row["Counter_Value"])
steps = agg["SQ_WAVES"] * 1000 / 1.0
print(sys.argv[2], "per chain-step: LDS conflict cycles %.1f, LDS instrs %.1f, VALU %.1f" % (
    agg["SQ_LDS_BANK_CONFLICT"] / steps, agg["SQ_INSTS_LDS"] / steps, agg["SQ_INSTS_VALU"] / steps))
PY
done
