#!/usr/bin/env python3
"""Fixed cost of one KernelWrapperSeeded call (the drop-in entry point on host buffers): the
median wall time of repeated calls at 0 MH steps (room upload, chain setup, the final pass, the
copy back, teardown) and at the config's step count, for config 2's and config 3's shapes.
Run on the GPU box (optionally under `rocprofv3 --hip-trace --stats` to see which HIP calls
the fixed cost is made of):  python tools/wrapper_overhead.py [reps]"""
import ctypes as C
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as graft  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    mh = graft.load_package()
    lib = mh.load_library()
    for n, chains, iters in ((8, 1024, 0), (8, 1024, 2000), (64, 65536, 0)):
        room = mh.synthetic_room(n)
        g = mh.abi.gpuConfig(chains, 0, 64, 0, 0, iters)
        walls = []
        for k in range(reps + 1):
            t0 = time.perf_counter()
            res = lib.KernelWrapperSeeded(*room.args(), C.byref(g), C.c_uint64(42 + k))
            w = time.perf_counter() - t0
            assert res, mh.last_error(lib)
            lib.KernelFreeResult(res)
            if k:  # (the first call pays module loading)
                walls.append(w)
        med = statistics.median(walls)
        print(json.dumps({"objects": n, "chains": chains, "iterations": iters,
                          "median_wall_ms": med * 1e3, "min_wall_ms": min(walls) * 1e3,
                          "chain_steps_per_s": chains * iters / med if iters else None}),
              flush=True)


if __name__ == "__main__":
    main()
