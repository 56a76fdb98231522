#!/usr/bin/env python3
"""Finds chains whose Accept draws u == 1.0f against an uphill proposal (Kernel.cu:706-713).

Accept takes u < min(1, (float)exp(BETA (star - cur))): for an uphill proposal the threshold
is exactly 1, so u == 1.0f -- the top value of the (0, 1] uniform, drawn when the Philox word is
>= 2^32 - 128 (about 3e-8 per word) -- rejects it. The rejection bound's certain-accept test
once took those proposals anyway (round 2; tools/bound_check.py found it), so the edge gets a
searched fixture, like the index-n pick (find_index_n.py).

The search scans the Philox words of chains 0..CHAINS-1 (seed SEED, subsequence = global chain
id) for a word >= 0xFFFFFF80 among the first WORDS, runs the oracle on those chains with its
u == 1.0f uphill counter (orc_u1_uphill_draws), and keeps the shortest run containing the event.
The result goes into tests/golden/golden.json under "u1_accept" (this script only adds that key).

Run from the repo root:  python tests/golden/find_u1_accept.py
"""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as graft  # noqa: E402

SEED, CHAINS, WORDS, KEEP = 42, 1 << 18, 6000, 2


def high_words(lib, seed, chain):
    buf = (C.c_uint32 * WORDS)()
    lib.orc_philox_stream(seed, chain, buf, WORDS)
    w = np.frombuffer(buf, dtype=np.uint32)
    return np.flatnonzero(w >= 0xFFFFFF80)


def search(mh, orc, lib, n):
    room = mh.synthetic_room(n)
    found = []
    orc.set_step_offlimits(False)
    for cid in range(CHAINS):
        hits = high_words(lib, SEED, cid)
        if hits.size == 0:
            continue
        steps = int(hits[-1]) // 3 + 10  # (a step draws ~4-5 words)
        orc.u1_uphill_draws(reset=True)
        orc.run_chains(room, 1, steps, SEED, chain_begin=cid)
        if orc.u1_uphill_draws() == 0:
            continue
        lo, hi = 1, steps
        while lo < hi:
            mid = (lo + hi) // 2
            orc.u1_uphill_draws(reset=True)
            orc.run_chains(room, 1, mid, SEED, chain_begin=cid)
            if orc.u1_uphill_draws() > 0:
                hi = mid
            else:
                lo = mid + 1
        print(f"N={n} chain {cid}: u == 1.0f against an uphill proposal at step {lo}", flush=True)
        found.append({"room": "synthetic", "n": n, "seed": SEED, "chain": cid,
                      "step": lo, "steps": lo + 40})
        if len(found) >= KEEP:
            break
    orc.set_step_offlimits(True)
    return found


def main():
    mh, orc = graft.load_package(), graft.load_oracle()
    lib = orc.load()
    found = search(mh, orc, lib, 8) + search(mh, orc, lib, 64)
    path = Path(__file__).with_name("golden.json")
    g = json.loads(path.read_text())
    g["u1_accept"] = found
    path.write_text(json.dumps(g, indent=1) + "\n")
    print("wrote", path, len(found), "cases")


if __name__ == "__main__":
    main()
