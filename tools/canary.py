#!/usr/bin/env python3
"""Short GPU canary run before a test suite: one small session per step kernel (full and
incremental, one chain per wavefront and several), each checked against the oracle. Meant to
run under `timeout` so a kernel that never finishes ends the GPU call early."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402

import __graft_entry__ as graft  # noqa: E402

mh, orc = graft.load_package(), graft.load_oracle()
for n, delta, lanes, chains, steps in [(64, "0", "", 64, 300), (256, "1", "", 8, 100),
                                       (64, "1", "", 32, 300), (20, "0", "32", 64, 300)]:
    os.environ["MH_DELTA"] = delta
    if lanes:
        os.environ["MH_LANES"] = lanes
    t0 = time.time()
    room = mh.synthetic_room(n)
    with mh.Session(room, chains, seed=5) as s:
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
        kind = s.step_kernel()
    rp, rc, _ = orc.run_chains(room, chains, steps, 5, threads=8)
    same = np.array_equal(pts.view(np.uint32), rp.view(np.uint32)) and np.array_equal(
        costs.view(np.uint32), rc.view(np.uint32))
    print(f"canary N={n} {kind}: bit-identical={same} ({time.time() - t0:.1f} s)", flush=True)
    os.environ.pop("MH_LANES", None)
    if not same:
        sys.exit(1)
