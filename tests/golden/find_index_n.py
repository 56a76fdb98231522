#!/usr/bin/env python3
"""Finds chains whose object pick draws index nObjs early (Kernel.cu:566-574, :598-602).

generateRandomIntInRange(n-1, 0) truncs (float)(u * (n - 1 + 0.999999)); for n >= 64 the float
product of u == 1.0f rounds up to n, an index one past the last object. The defined semantics
 redraw it like a frozen pick. A draw is 1.0f when its Philox word is >= 2^32 -
128, about 3e-8 per word, so the edge needs a searched fixture to be exercised in a short run.

The search scans the Philox words of chains 0..CHAINS-1 (seed SEED, subsequence = global chain
id, rocRAND layout) for a word >= 0xFFFFFF80 among the first WORDS, then runs the oracle on the
candidates and keeps those whose pick actually drew index n (orc_index_n_draws). The result is
written into tests/golden/golden.json under "index_n" (run make_golden.py first; this script
only adds that key).

Run from the repo root:  python tests/golden/find_index_n.py
"""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as graft  # noqa: E402

N, SEED, CHAINS, WORDS, KEEP = 64, 42, 1 << 17, 1600, 3


def first_high_word(lib, seed, chain):
    buf = (C.c_uint32 * WORDS)()
    lib.orc_philox_stream(seed, chain, buf, WORDS)
    w = np.frombuffer(buf, dtype=np.uint32)
    hit = np.flatnonzero(w >= 0xFFFFFF80)
    return int(hit[0]) if hit.size else -1


def main():
    mh, orc = graft.load_package(), graft.load_oracle()
    lib = orc.load()
    room = mh.synthetic_room(N)
    found = []
    for cid in range(CHAINS):
        d = first_high_word(lib, SEED, cid)
        if d < 0:
            continue
        # draws per step are ~4-5 words: run a little past the candidate word
        steps = d // 3 + 10
        orc.index_n_draws(reset=True)
        orc.run_chains(room, 1, steps, SEED, chain_begin=cid)
        hits = orc.index_n_draws()
        if hits == 0:
            continue
        # the shortest run that contains the redraw
        lo, hi = 1, steps
        while lo < hi:
            mid = (lo + hi) // 2
            orc.index_n_draws(reset=True)
            orc.run_chains(room, 1, mid, SEED, chain_begin=cid)
            if orc.index_n_draws() > 0:
                hi = mid
            else:
                lo = mid + 1
        print(f"chain {cid}: word {d} >= 0xFFFFFF80, index-n pick at step {lo}")
        found.append({"room": "synthetic", "n": N, "seed": SEED, "chain": cid,
                      "first_step": lo, "steps": lo + 50})
        if len(found) >= KEEP:
            break
    path = Path(__file__).with_name("golden.json")
    g = json.loads(path.read_text())
    g["index_n"] = found
    path.write_text(json.dumps(g, indent=1) + "\n")
    print("wrote", path, len(found), "cases")


if __name__ == "__main__":
    main()
