#!/usr/bin/env python3
"""Per-phase cycle shares of the step kernel from a diagnostic build with MH_STAMPS=1
(abvar/libmhgpu_stamps.so, made by tools/build_ablate.sh stamps). Run on the GPU box:
    MH_LANES=32 python tools/stamps.py [objects] [chains] [iters]
Read the SHARES, not the absolute time: the stamps' waits forbid some overlap."""
import ctypes as C
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("MH_LIB", str(ROOT / "abvar" / "libmhgpu_stamps.so"))
import __graft_entry__ as graft  # noqa: E402

DELTA_PHASES = ["propose+objects", "clearance delta", "relationships", "symmetry delta",
                "bound + term lists", "replay", "accept/restore", "(replay: dense part)"]
SPEC_PHASES = ["tree + record count", "apply", "views barrier (wait for wave 1)",
               "jobs (exact terms)", "own ordered sums", "bound (estimates, parts)",
               "sums barrier (wait for wave 1)",
               "costs + accept + commit", "", "", "", ""]
PHASES = ["propose", "A per-object", "B symmetry", "C clearance pairs", "D reject bound",
          "E SA walk + CL list", "F PW/ANG + replay", "accept/undo"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    chains = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    mh = graft.load_package()
    lib = mh.load_library()
    with mh.Session(mh.synthetic_room(n), chains, seed=42) as s:
        lanes, cpw, s_kind = s.step_kernel()
        print(f"[stamps] session created: {lanes} lanes/chain, {cpw} chains/workgroup, {s_kind}",
              flush=True)
        s.run(0)
        s.current_costs()  # (synchronises the set-up)
        t0 = time.perf_counter()
        s.run(iters)
        s.current_costs()  # (synchronises)
        wall = time.perf_counter() - t0
        print(f"[stamps] run: {wall * 1e3:.3f} ms wall for {iters} steps", flush=True)
        s.finalize()
        print("[stamps] finalize launched", flush=True)
        acc_rate = s.summary().accepted / float(chains * iters)
    if hasattr(lib, "mh_debug_check"):  # MH_CHECK builds: the first index violation, if any
        ck = (C.c_uint * 8)()
        assert lib.mh_debug_check(ck) == 0
        print(f"[check] violations={ck[0]} first site={ck[1]} values=({ck[2]}, {ck[3]}) "
              f"wave={ck[4]}", flush=True)
    out = (C.c_ulonglong * 16)()
    if not hasattr(lib, "mh_debug_phase_cycles"):  # (a library without stamps: the wall time only)
        return
    if s_kind == "speculative":  # one chain per wavefront, per-batch phases
        assert lib.mh_debug_spec_cycles(out) == 0
        tot = sum(out[:8])  # ([8] loop cycles, [9] its 100 MHz ticks, [12]-[15] counts)
        batches, steps = out[14], out[15]
        print(f"N={n} chains={chains} iters={iters} speculative acceptance={acc_rate:.4f} "
              f"steps per batch {steps / max(1, batches):.3f}; batches: {batches} "
              f"(exact {out[13]}, of them refresh {out[12]}); shader clock over the loop "
              f"{out[8] / max(1, out[9]) * 0.1:.3f} GHz (s_memtime / s_memrealtime)")
        for name, v in zip(SPEC_PHASES, out[:8]):
            if not name:
                continue
            print(f"  {name:24s} {100.0 * v / tot:6.2f}%   {v / max(1, batches):10.1f} cycles/batch"
                  f"   {v / max(1, steps):10.1f} cycles/step")
        return
    delta = hasattr(lib, "mh_debug_delta_cycles") and s_kind == "incremental"
    if delta:  # incremental step kernel: per-wavefront stamps, 64/lanes chains per wavefront
        assert lib.mh_debug_delta_cycles(out) == 0
        names, per = DELTA_PHASES, chains * iters / (64 // lanes)
        unit = "cycles/wave-step"
    else:
        assert lib.mh_debug_phase_cycles(out) == 0
        names, per, unit = PHASES, chains * iters, "cycles/chain-step"
    tot = sum(out[:7] if delta else out[:8])  # (delta: [7] is a part of [5])
    print(f"N={n} chains={chains} iters={iters} lanes/chain={lanes} delta={delta} "
          f"acceptance={acc_rate:.4f}")
    for name, v in zip(names, out[:8]):
        print(f"  {name:18s} {100.0 * v / tot:6.2f}%   {v / per:10.1f} {unit}")
    if not delta and out[8]:
        steps = chains * iters
        print(f"  rejection bound evaluated on {out[8] / steps:.4f} of steps, certain reject on "
              f"{out[9] / steps:.4f} ({out[9] / out[8]:.4f} of those evaluated), certain accept "
              f"on {out[10] / steps:.4f}; exact costs of the current configuration recomputed on "
              f"{out[11] / steps:.4f}")
    if not delta and out[13]:  # the loop's shader cycles and 100 MHz ticks, summed over chains
        print(f"  shader clock over the step loop {out[12] / out[13] * 0.1:.3f} GHz "
              f"(s_memtime / s_memrealtime)")
    if delta and out[12]:  # counts (MH_STAMPS=2 builds): per step that reached the replay
        steps = chains * iters
        rep = max(1, out[12] - out[13] - out[14])
        print(f"  rejection bound evaluated on {out[12] / steps:.4f} of steps, certain reject on "
              f"{out[13] / steps:.4f}, certain accept on {out[14] / steps:.4f}; exact costs of the "
              f"current configuration recomputed on {out[15] / steps:.4f}; per replayed step: "
              f"mean Clearance list "
              f"{out[8] / rep:.2f}, SurfaceArea list {out[9] / rep:.2f}, overflow fractions "
              f"{out[10] / rep:.4f} / {out[11] / rep:.4f}")


if __name__ == "__main__":
    main()
