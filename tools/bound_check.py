#!/usr/bin/env python3
"""Verifies every decision the rejection bound takes, on real chains: the MH_CHECK build
(metropolis-hastings-gpgpu_amd/libmhgpu_check.so, made by __graft_entry__.build()) also computes the exact costs of every
proposal the bound decided and checks that the exact total lies in the bound's interval, that
the current total lies in the interval it carries, and that a certain REJECT / ACCEPT is
Accept's own decision (Kernel.cu:706-713); the first violation is recorded.
    python tools/bound_check.py [--quick]      (on the GPU box; prints one line per case)"""
import ctypes as C
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LIB = Path(os.environ.get("MH_CHECK_LIB", ROOT / "metropolis-hastings-gpgpu_amd" /
                         "libmhgpu_check.so"))  # (__graft_entry__.build())
SITES = {20: "certain REJECT but Accept accepts", 21: "certain ACCEPT but Accept rejects",
         22: "exact total outside the bound's interval",
         23: "current total outside the carried interval",
         24: "exact pass of the current configuration differs from the carried total",
         25: "exact total against the current interval decided wrongly",
         26: "a launch ended without the current configuration's exact costs",
         27: "cached Clearance row sums differ from a fresh build",
         28: "cached Clearance column sum differs from a fresh one",
         29: "cached SurfaceArea sums differ from a fresh build",
         30: "a FocalPoint estimate outside kDeltaCph",
         31: "a PairWise estimate outside kPwEstU U",
         32: "a PairWiseAngle estimate outside its allowance",
         33: "a deferred Symmetry row maximum outside its estimate's allowance",
         14: "the final pass's output slot outside [0, n_chains)",
         16: "the final pass's OffLimits boxes outside the chain's LDS slot"}

# (room kind, N, chains, steps, kernel): the configs' rooms and edge rooms; "wild" moves every
# object far outside the proven symmetry range, "negw" flips the weights' signs.
CASES = [("syn", 64, 8192, 2000, "full"), ("syn", 256, 2048, 1500, "incremental"),
         ("syn", 8, 1024, 5000, "full"), ("syn", 100, 2048, 1500, "full"),
         ("syn", 100, 2048, 1500, "incremental"), ("syn", 160, 1024, 1000, "incremental"),
         ("wrap", 64, 2048, 2000, "full"), ("manyrel", 200, 1024, 1000, "incremental"),
         ("wrap", 256, 1024, 1000, "incremental"),
         ("negw", 64, 2048, 2000, "full"), ("negw", 256, 1024, 1000, "incremental"),
         ("wild", 64, 1024, 1000, "full"), ("wild", 256, 512, 500, "incremental"),
         # the round-5 download fault's test shape (test_bound_decision_paths[main-32]): the
         # console harness's room, current costs read, then the final pass (index-checked)
         ("main", 32, 512, 600, "full"), ("main", 32, 512, 600, "incremental"),
         # the speculative kernel's instance that decides on the bound (mh_spec.hip: nodes'
         # bounds against their exact costs, at every node of every batch): config 2's room, a
         # wrapped one, negated weights, poses far outside the symmetry range; 16- and 8-node trees
         ("syn", 8, 256, 3000, "speculative"), ("syn", 8, 1024, 3000, "speculative-h1"),
         ("wrap", 8, 512, 2000, "speculative"), ("negw", 8, 512, 2000, "speculative"),
         ("wild", 8, 256, 1000, "speculative")]


def room_of(mh, kind, n):
    if kind == "manyrel":  # more relationships than objects (R > N + 1)
        return mh.synthetic_room(n, n_rel=3 * n + 5)
    if kind == "main":
        return mh.main_fixture()
    room = mh.synthetic_room(n)
    if kind == "wrap":  # angle ranges crossing zero: the fmodf branch of Kernel.cu:245-250
        for k in range(room.srf.nRelationships):
            room.rsa[k].angleMin = 7 * 3.1416 / 4
            room.rsa[k].angleMax = 3.1416 / 4
    if kind == "negw":
        for f in ("WeightPairWise", "WeightVisualBalance", "WeightSymmetry", "WeightClearance"):
            setattr(room.srf, f, -getattr(room.srf, f))
    if kind == "wild":
        for i in range(n):
            room.cfg[i].x *= 3.0e15
            room.cfg[i].y *= -2.0e15
    return room


def one(kind, n, chains, steps, kernel):
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as graft
    mh = graft.load_package()
    os.environ["MH_DELTA"] = "1" if kernel == "incremental" else "0"
    os.environ["MH_SPEC"] = "1" if kernel.startswith("speculative") else "0"
    os.environ["MH_SPEC_BOUND"] = "1"
    os.environ["MH_SPEC_H"] = "1" if kernel.endswith("-h1") else ""
    kernel = kernel.split("-")[0]
    lib = mh.load_library(str(LIB))
    mh.abi._lib = lib  # the Session wrapper uses the module's library
    room = room_of(mh, kind, n)
    with mh.Session(room, chains, seed=4242 + n) as s:
        assert s.step_kernel()[2].split("-")[0] == kernel, s.step_kernel()
        s.run(steps)
        s.current_costs()
        s.finalize()
        _, costs = s.download()
    ck = (C.c_uint * 8)()
    fn = {"incremental": lib.mh_debug_check_delta,
          "speculative": lib.mh_debug_check_spec}.get(kernel, lib.mh_debug_check)
    assert fn(ck) == 0
    if kernel != "full":  # (the init and final passes are the full kernel's: its record)
        ckf = (C.c_uint * 8)()
        assert lib.mh_debug_check(ckf) == 0
        if ckf[0] and not ck[0]:
            ck[0], ck[1], ck[2], ck[3] = ckf[0], ckf[1], ckf[2], ckf[3]
    if kernel == "speculative" and ck[0]:
        import struct
        g = (C.c_uint * 12)()
        assert lib.mh_debug_spec_ck(g) == 0
        f = lambda v: struct.unpack("f", struct.pack("I", v))[0]
        print(f"[spec-ck] sc={f(g[1])!r} t={f(g[2])!r} e={f(g[3])!r} cur={f(g[4])!r} u={f(g[5])!r} "
              f"d={g[6] & 255} node={(g[6] >> 8) & 255} dep={g[6] >> 16} cpar={g[7] & 255} "
              f"kb={(g[7] >> 8) & 255} H={g[7] >> 16} cur0={f(g[8])!r} done={g[9]} e0={f(g[10])!r} "
              f"hf={g[11]}", flush=True)
    dc = (C.c_ulonglong * 4)()
    fd = {"incremental": lib.mh_debug_decisions_delta,
          "speculative": lib.mh_debug_decisions_spec}.get(kernel, lib.mh_debug_decisions)
    assert fd(dc) == 0
    steps_all = float(chains * steps)
    rates = (f"; of {chains * steps} steps: certain reject {dc[1] / steps_all:.4f}, certain "
             f"accept {dc[2] / steps_all:.4f}, open {(dc[0] - dc[1] - dc[2]) / steps_all:.4f}, "
             f"exact current pass {dc[3] / steps_all:.4f}") if dc[0] else ""
    site = SITES.get(ck[1], str(ck[1]))
    # (speculative: decisions at every evaluated node, the realised path's and the others')
    print(f"[bound] {kind} N={n} {kernel}: {chains} x {steps} steps, {ck[5]} bound decisions "
          f"checked, violations {ck[0]}" + (f" (first: {site}, values {ck[2]:#x} {ck[3]:#x})"
                                            if ck[0] else "") + rates, flush=True)
    return ck[0] == 0


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        kind, n, chains, steps, kernel = sys.argv[2], *map(int, sys.argv[3:6]), sys.argv[6]
        sys.exit(0 if one(kind, n, chains, steps, kernel) else 1)
    quick = "--quick" in sys.argv
    ok = True
    for kind, n, chains, steps, kernel in CASES:
        if quick:
            chains, steps = max(64, chains // 8), max(200, steps // 4)
        rc = subprocess.run([sys.executable, __file__, "--one", kind, str(n), str(chains),
                             str(steps), kernel], timeout=300).returncode
        ok &= rc == 0
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
