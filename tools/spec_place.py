#!/usr/bin/env python3
"""Where and when the speculative kernel's chains ran, from the stamps build
(abvar/libmhgpu_stamps.so, tools/build_ablate.sh stamps): per chain of the last launch, its
loop's start and end on the constant 100 MHz counter and its CU (HW_ID / XCC_ID). Shows whether
every chain was resident from the start (a launch's time = one chain's) or some waited for a
slot, and how many chains each CU held. Run on the GPU box:
    MH_LIB=abvar/libmhgpu_stamps.so python tools/spec_place.py [objects] [chains] [iters]"""
import ctypes as C
import os
import sys
from collections import Counter
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("MH_LIB", str(ROOT / "abvar" / "libmhgpu_stamps.so"))
import __graft_entry__ as graft  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    chains = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    mh = graft.load_package()
    lib = mh.load_library()
    with mh.Session(mh.synthetic_room(n), chains, seed=42) as s:
        lanes, cpw, kind = s.step_kernel()
        occ = s.occupancy()
        s.run(iters)  # (warm-up launch)
        s.current_costs()
        s.run(iters)
        s.current_costs()
    m = min(chains, 16384)
    buf = (C.c_ulonglong * (6 * 16384))()
    assert lib.mh_debug_spec_place(buf) == 0
    t0 = [buf[6 * i] for i in range(m)]
    t1 = [buf[6 * i + 1] for i in range(m)]
    hw = [buf[6 * i + 2] for i in range(m)]
    nb = [buf[6 * i + 3] for i in range(m)]
    ne = [buf[6 * i + 4] for i in range(m)]
    nr = [buf[6 * i + 5] for i in range(m)]
    base = min(t0)
    dur = [(b - a) / 100.0 for a, b in zip(t0, t1)]  # microseconds
    start = [(a - base) / 100.0 for a in t0]
    end = [(b - base) / 100.0 for b in t1]
    span = max(end)

    def cu_of(h):
        lo, xcc = h & 0xFFFFFFFF, h >> 32
        return (xcc & 0xF, (lo >> 13) & 0x7, (lo >> 12) & 1, (lo >> 8) & 0xF)

    per_cu = Counter(cu_of(h) for h in hw)
    late = sum(1 for x in start if x > 0.1 * span)
    print(f"N={n} chains={chains} {kind} ({lanes} lanes per chain, occupancy {occ} chains per CU), "
          f"last launch of {iters} steps")
    print(f"  launch span {span:.1f} us; chain loop duration min {min(dur):.1f} / mean "
          f"{sum(dur) / m:.1f} / max {max(dur):.1f} us; chains starting after 10% of the span: "
          f"{late}; last start {max(start):.1f} us")
    hist = Counter(per_cu.values())
    print(f"  CUs used {len(per_cu)}; chains per CU: "
          + ", ".join(f"{k}: {v} CUs" for k, v in sorted(hist.items())))
    # duration by how many chains shared the CU
    by = {}
    for h, d in zip(hw, dur):
        by.setdefault(per_cu[cu_of(h)], []).append(d)
    # the slowest and fastest tenth of the chains: batches, exact and refresh batches
    order = sorted(range(m), key=lambda i: dur[i])
    for name, sel in (("fastest tenth", order[: m // 10]), ("median tenth", order[m * 9 // 20: m * 11 // 20]),
                      ("slowest tenth", order[-(m // 10):])):
        k = len(sel)
        print(f"  {name:14s} duration {sum(dur[i] for i in sel) / k:8.1f} us, batches "
              f"{sum(nb[i] for i in sel) / k:8.1f}, exact {sum(ne[i] for i in sel) / k:7.1f}, "
              f"refresh {sum(nr[i] for i in sel) / k:7.1f}, us per batch "
              f"{sum(dur[i] / max(1, nb[i]) for i in sel) / k:.3f}")
    print("  slowest chains (us, batches, exact, refresh): " + "; ".join(
        f"{i}: {dur[i]:.0f}, {nb[i]}, {ne[i]}, {nr[i]}" for i in order[-8:][::-1]))
    # the SIMDs of the chain's wavefronts (HW_ID bits 5:4), and the waves of this launch per SIMD
    sb = (C.c_uint * (4 * 16384))()
    assert lib.mh_debug_spec_simd(sb) == 0
    wpc = lanes // 64
    simd = [[(sb[4 * i + w] >> 4) & 3 for w in range(wpc)] for i in range(m)]
    per_simd = Counter()
    for i in range(m):
        for w in range(wpc):
            per_simd[cu_of(hw[i]) + (simd[i][w],)] += 1
    print("  wavefronts per SIMD: " + ", ".join(f"{k}: {v} SIMDs" for k, v in
                                                 sorted(Counter(per_simd.values()).items())))
    shared = [i for i in range(m) if len(set(simd[i])) < wpc]
    print(f"  chains whose wavefronts share a SIMD: {len(shared)} of {m}")
    # a chain's time against its wavefronts' SIMD loads (the most crowded of its SIMDs)
    load = {}
    for i in range(m):
        worst = max(per_simd[cu_of(hw[i]) + (sd,)] for sd in simd[i])
        key = (len(set(simd[i])) < wpc, worst)
        load.setdefault(key, []).append(dur[i])
    for (sh, worst), v in sorted(load.items()):
        print(f"    {'shared' if sh else 'apart '} SIMD, most crowded SIMD {worst} waves: "
              f"{len(v)} chains, mean {sum(v) / len(v):.1f} us, max {max(v):.1f} us")
    print("  mean chain duration by chains on its CU: "
          + ", ".join(f"{k}: {sum(v) / len(v):.1f} us" for k, v in sorted(by.items())))


if __name__ == "__main__":
    main()
