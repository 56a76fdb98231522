#!/usr/bin/env python3
"""Diagnostic: per chain, the first step count k at which the speculative kernel's accepted
count or carried costs differ from the oracle's (1-chain sessions)."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as graft  # noqa: E402

os.environ["MH_SPEC"] = "1"
mh, orc = graft.load_package(), graft.load_oracle()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
kmax = int(sys.argv[2]) if len(sys.argv) > 2 else 60
room = mh.synthetic_room(n)
seed = 5150
orc.set_step_offlimits(False)
for c in range(4):
    for k in range(1, kmax + 1):
        with mh.Session(room, 1, seed=seed, chain_offset=c) as s:
            s.run(k)
            cur = s.current_costs()[0]
            acc = s.summary().accepted
            s.finalize()
            pts, costs = s.download()
        rp, rc, ra = orc.run_chains(room, 1, k, seed, chain_begin=c)
        same = (np.array_equal(pts.view(np.uint32), rp.view(np.uint32)) and
                np.array_equal(cur[:6].view(np.uint32), rc[0, :6].view(np.uint32)))
        if not same or acc != int(ra[0]):
            print(f"chain {c}: first difference at k={k}: acc dev {acc} ref {int(ra[0])}; "
                  f"cur dev {cur} ref {rc[0]}; pts dev {pts[0, :, [0, 1, 4]].T.tolist()} "
                  f"ref {rp[0, :, [0, 1, 4]].T.tolist()}", flush=True)
            # the previous state and the proposal the oracle draws at step k
            rs, rcs, _ = orc.run_chains(room, 1, k - 1, seed, chain_begin=c, state=True)
            print(f"   state before: {rs[0][:, [0, 1, 4]].tolist()} costs {rcs[0]}", flush=True)
            break
    else:
        print(f"chain {c}: identical through k={kmax}", flush=True)
