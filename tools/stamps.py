#!/usr/bin/env python3
"""Per-phase cycle shares of the step kernel from a diagnostic build with MH_STAMPS=1
(ablate/libmhgpu_stamps.so, made by tools/build_ablate.sh stamps). Run on the GPU box:
    MH_LANES=32 python tools/stamps.py [objects] [chains] [iters]
Read the SHARES, not the absolute time: the stamps' waits forbid some overlap."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("MH_LIB", str(ROOT / "ablate" / "libmhgpu_stamps.so"))
import __graft_entry__ as graft  # noqa: E402

PHASES = ["propose", "A per-object", "B symmetry", "C ordered sums", "D surface area",
          "E clearance", "F pairwise/angle", "accept/undo"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    chains = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    mh = graft.load_package()
    lib = mh.load_library()
    with mh.Session(mh.synthetic_room(n), chains, seed=42) as s:
        s.run(iters)
        s.finalize()
        s.summary()
        lanes, cpw = s.geometry()
    out = (C.c_ulonglong * 8)()
    assert lib.mh_debug_phase_cycles(out) == 0
    tot = sum(out)
    print(f"N={n} chains={chains} iters={iters} lanes/chain={lanes}")
    for name, v in zip(PHASES, out):
        print(f"  {name:18s} {100.0 * v / tot:6.2f}%   {v / (chains * iters):10.1f} cycles/chain-step")


if __name__ == "__main__":
    main()
