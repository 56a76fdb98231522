#!/usr/bin/env python3
"""End-to-end rate of the drop-in entry point: KernelWrapperSeeded on host buffers, as the
reference's caller uses it (room upload, chain setup, sampling, final pass, and the copy of
every chain's points and costs back to host memory), for config 3's shape. Run on the GPU box:
    python tools/e2e_wrapper.py [iterations] [chains]
Prints one JSON line; DESIGN.md quotes it next to bench.py's device-resident rate."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as graft  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    chains = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    mh = graft.load_package()
    lib = mh.load_library()
    room = mh.synthetic_room(64)
    g = mh.abi.gpuConfig(chains, 0, 64, 0, 0, iters)
    warm = mh.abi.gpuConfig(chains, 0, 64, 0, 0, 10)
    res = lib.KernelWrapperSeeded(*room.args(), C.byref(warm), C.c_uint64(1))
    assert res, mh.last_error(lib)
    lib.KernelFreeResult(res)
    t0 = time.perf_counter()
    res = lib.KernelWrapperSeeded(*room.args(), C.byref(g), C.c_uint64(42))
    wall = time.perf_counter() - t0
    assert res, mh.last_error(lib)
    lib.KernelFreeResult(res)
    print(json.dumps({"entry": "KernelWrapperSeeded", "objects": 64, "chains": chains,
                      "iterations": iters, "wall_s": wall,
                      "chain_steps_per_s": chains * iters / wall,
                      "result_bytes": chains * (64 * 24 + 40)}))


if __name__ == "__main__":
    main()
