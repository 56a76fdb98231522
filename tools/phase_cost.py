#!/usr/bin/env python3
"""Per-phase costs per chain-step from tools/phase_cost_box.sh output:
    python tools/phase_cost.py gpurun_out/<tag> [--chains 65536] [--iters 1000]"""
import argparse
import csv
import glob
import os
from collections import defaultdict

NAMES = {"2": "ablate per-object atan2/cos", "16": "ablate PW/ANG terms", "dbl1": "A per-object",
         "dbl2": "B full symmetry", "dbl64": "B delta symmetry",
         "dbl4": "E surface area walk", "dbl8": "E clearance",
         "dbl16": "F pairwise appends", "dbl32": "G replay",
         "dbl128": "C clearance pair update", "dbl256": "D bound terms + sums"}


def load(d, kernel):
    per = defaultdict(list)
    dur = []
    for row in csv.DictReader(open(os.path.join(d, "pmc_counter_collection.csv"))):
        if kernel in row["Kernel_Name"]:
            per[row["Counter_Name"]].append(float(row["Counter_Value"]))
            dur.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    c = {k: sum(v) / len(v) for k, v in per.items()}
    c["ns"] = sum(dur) / max(len(dur), 1)
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag_dir")
    ap.add_argument("--kernel", default="mh_kernel<64, 1, 1>")
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=1000)
    a = ap.parse_args()
    steps = a.chains * a.iters
    base = load(os.path.join(a.tag_dir, "pmc_0"), a.kernel)
    keys = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
            "SQ_ACTIVE_INST_VALU", "ns"]
    keys = [k for k in keys if k in base]
    hdr = f"{'phase':28s}" + "".join(f"{k.replace('SQ_INSTS_', '').replace('SQ_ACTIVE_INST_', 'act_').replace('SQ_LDS_BANK_CONFLICT', 'ldsconf'):>11s}" for k in keys)
    print(hdr)
    print(f"{'whole step':28s}" + "".join(f"{base[k] / (steps if k != 'ns' else 1):11.1f}" for k in keys))
    # probe builds (dblK: phase run twice, +cost) and ablations (K: phase compiled out, -cost)
    for d in sorted(glob.glob(os.path.join(a.tag_dir, "pmc_*"))):
        v = os.path.basename(d)[4:]
        if not os.path.isdir(d) or v == "0":
            continue
        c = load(d, a.kernel)
        sign = 1.0 if v.startswith("dbl") else -1.0
        print(f"{NAMES.get(v, v):28s}" + "".join(
            f"{sign * (c[k] - base[k]) / (steps if k != 'ns' else 1):11.1f}" for k in keys))


if __name__ == "__main__":
    main()
