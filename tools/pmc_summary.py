#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes written by tools/profile_box.sh.

    python tools/pmc_summary.py gpurun_out/<tag> [--kernel SUBSTR] [--chains N] [--json OUT]

Prints, per kernel (default: the chain step kernel), the per-dispatch mean of every counter
collected, plus derived figures. HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so the
read side is doubled (an upper bound for narrower accesses). --json writes the traffic record
bench.py reads (profiles/pmc_step_kernel.json).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(tag_dir, kernel_substr):
    per = defaultdict(list)  # counter -> values (one per dispatch)
    meta = {}
    for f in glob.glob(os.path.join(tag_dir, "pmc_*", "pmc_counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_substr not in row["Kernel_Name"]:
                    continue
                per[row["Counter_Name"]].append(float(row["Counter_Value"]))
                meta = {k: row[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size",
                                            "LDS_Block_Size", "VGPR_Count", "SGPR_Count",
                                            "Scratch_Size")}
                meta["duration_ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    return {k: sum(v) / len(v) for k, v in per.items()}, meta


def _srchash(tag_dir):
    p = os.path.join(tag_dir, "srchash")
    return open(p).read().strip() if os.path.exists(p) else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag_dir")
    ap.add_argument("--kernel", default="mh_kernel<64, 1, 1>")
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=1000, help="MH steps per launch")
    ap.add_argument("--json", default=None)
    ap.add_argument("--profile", default=None,
                    help="the tracked profiles/ copy of this summary (recorded in the JSON)")
    a = ap.parse_args()
    c, meta = load(a.tag_dir, a.kernel)
    if not c:
        raise SystemExit(f"no dispatches of {a.kernel!r} under {a.tag_dir}")
    print(json.dumps(meta))
    for k in sorted(c):
        print(f"{k:28s} {c[k]:.6g}")
    d = {}
    if "SQ_WAVE_CYCLES" in c and "SQ_ACTIVE_INST_VALU" in c:
        d["valu_active_frac_of_wave_cycles"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
    if "GRBM_GUI_ACTIVE" in c:
        simd_cycles = 1024.0 * c["GRBM_GUI_ACTIVE"] / 8.0
        d["kernel_cycles_per_xcd"] = c["GRBM_GUI_ACTIVE"] / 8.0
        if "SQ_INSTS_VALU" in c:
            d["valu_issue_util_flat"] = 2.0 * c["SQ_INSTS_VALU"] / simd_cycles
            extra = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                     "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_TRANS_F64")
            if all(k in c for k in extra):
                busy = 2.0 * c["SQ_INSTS_VALU"] + 2.0 * (
                    c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] +
                    c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_CVT"] +
                    c["SQ_INSTS_VALU_TRANS_F32"]) + 6.0 * c["SQ_INSTS_VALU_TRANS_F64"]
                d["valu_busy_simd_cycles"] = busy
                d["valu_issue_util"] = busy / simd_cycles
    if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
        d["wait_inst_any_frac"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
    if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c:
        d["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
    if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
        rd = 2.0 * c.get("FETCH_SIZE", 0.0) * 1024
        wr = c.get("WRITE_SIZE", 0.0) * 1024
        d["hbm_read_bytes_corrected"] = rd
        d["hbm_write_bytes"] = wr
        d["hbm_bytes_per_launch"] = rd + wr
    for k, v in d.items():
        print(f"{k:28s} {v:.6g}")
    if a.json and "hbm_bytes_per_launch" in d:
        rec = {"kernel": meta.get("Kernel_Name"), "chains_per_launch": a.chains,
               "hbm_bytes_per_launch": d["hbm_bytes_per_launch"],
               "fetch_size_kib": c.get("FETCH_SIZE"), "write_size_kib": c.get("WRITE_SIZE"),
               "correction": "read side = 2 x FETCH_SIZE (gfx950, MI355X_MICROARCH.md HBM)",
               "iters_per_launch": a.iters,
               "valu_wave_insts_per_launch": c.get("SQ_INSTS_VALU"),
               "salu_insts_per_launch": c.get("SQ_INSTS_SALU"),
               "valu_issue_util": d.get("valu_issue_util"),
               "valu_issue_util_flat": d.get("valu_issue_util_flat"),
               "valu_pricing": "2 cyc/VALU; +2 fp64 add/mul/fma, cvt, f32 trans; +6 f64 trans",
               "source": os.path.normpath(a.tag_dir), "profile": a.profile,
               # the profiled library's source hash (tools/profile_box.sh copied its .srchash):
               # bench.py uses this record only while the loaded library has the same one
               "srchash": _srchash(a.tag_dir)}
        with open(a.json, "w") as fh:
            json.dump(rec, fh, indent=1)
        print("wrote", a.json)


if __name__ == "__main__":
    main()
