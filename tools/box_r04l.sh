#!/bin/bash
# Round 4: the shared math's cost (A/B: round 3's library, the OCML ablation, the product) and
# the speculative kernel's issue counters at config 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04l; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_spec.log 2>&1 || { tail -40 $OUT/pytest_spec.log; exit 1; }
tail -1 $OUT/pytest_spec.log
MH_AB_REPS=2 MH_AB_CFGS="256,32768,1000,1 64,65536,1000,3 8,1024,2000,4" bash tools/box_abn.sh r04l/ab head ocml main || exit 1
ARGS="--objects 8 --chains 1024 --iters 2000 --steps 2 --warmup 1 --no-cpu-baseline --e2e-iters 0"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY \
    -d $OUT/pmc_spec -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_spec.log 2>&1 || { tail -5 $OUT/pmc_spec.log; exit 1; }
MH_SPEC=0 timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY \
    -d $OUT/pmc_few -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_few.log 2>&1 || { tail -5 $OUT/pmc_few.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for tag in ("spec", "few"):
    files = glob.glob(f"gpurun_out/r04l/pmc_{tag}/**/*counter_collection*.csv", recursive=True)
    agg = collections.defaultdict(float); n = collections.Counter()
    for f in files:
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            if "mh_spec_kernel" not in k and "mh_kernel" not in k: continue
            if "ILi64ELi1ELi4E" not in k and "spec" not in k: continue
            agg[row["Counter_Name"]] += float(row["Counter_Value"]); n[row["Counter_Name"]] += 1
    print(tag, {k: "%.4g" % v for k, v in sorted(agg.items())}, dict(n))
PY
