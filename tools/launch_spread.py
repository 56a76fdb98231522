#!/usr/bin/env python3
"""Why one step-kernel launch takes longer than another: per 1,000-step launch of one session,
its time (the product library, hipEvent-free wall time around a synchronised launch) beside what
the check build counted in the same launch of the same chains (libmhgpu_check.so: the bound's
decisions -- certain reject, certain accept, open -- and the exact passes of the current
configuration, mh_debug_decisions[_delta]). The two libraries run the same trajectories bit for
bit, so launch k of one is launch k of the other. Run on the GPU box:
    python tools/launch_spread.py [objects] [chains] [launches] [steps per launch]
Each library runs in a child process of its own (they export the same symbols)."""
import ctypes as C
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def child(which, n, chains, launches, iters):
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as graft
    mh = graft.load_package()
    lib = mh.load_library(str(mh.LIB_PATH.with_name("libmhgpu_check.so")) if which == "check"
                          else None)
    mh.abi._lib = lib
    rows = []
    with mh.Session(mh.synthetic_room(n), chains, seed=42) as s:
        kind = s.step_kernel()[2]
        delta = kind == "incremental"
        prev = [0, 0, 0, 0]
        s.run(0)
        s.current_costs()  # (synchronises the set-up)
        for k in range(launches):
            t0 = time.perf_counter()
            s.run(iters)
            s.current_costs()  # (synchronises)
            dt = time.perf_counter() - t0
            row = {"launch": k, "ms": dt * 1e3}
            if which == "check":
                dc = (C.c_ulonglong * 4)()
                f = lib.mh_debug_decisions_delta if delta else lib.mh_debug_decisions
                assert f(dc) == 0
                cur = list(dc)
                d = [cur[i] - prev[i] for i in range(4)]
                prev = cur
                steps = float(chains * iters)
                row.update(evaluated=d[0] / steps, reject=d[1] / steps, accept=d[2] / steps,
                           open=(d[0] - d[1] - d[2]) / steps, exact_current=d[3] / steps)
            rows.append(row)
    print(json.dumps({"which": which, "kind": kind, "rows": rows}))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2], *map(int, sys.argv[3:7]))
        return
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    chains = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
    launches = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 1000
    res = {}
    for which in ("product", "check"):
        out = subprocess.run([sys.executable, __file__, "--child", which, str(n), str(chains),
                              str(launches), str(iters)], capture_output=True, text=True,
                             timeout=600, env=dict(os.environ, MH_SPEC="0"))
        if out.returncode != 0:
            sys.exit(out.stdout[-2000:] + out.stderr[-3000:])
        res[which] = json.loads(out.stdout.strip().splitlines()[-1])
    print(f"N={n} chains={chains} {res['product']['kind']} kernel, {iters} steps per launch "
          f"(fractions of the launch's chain-steps; time from the product library)")
    print(f"{'launch':>6} {'ms':>9} {'reject':>8} {'accept':>8} {'open':>8} {'exact cur':>10}")
    for p, c in zip(res["product"]["rows"], res["check"]["rows"]):
        print(f"{p['launch']:>6} {p['ms']:>9.1f} {c['reject']:>8.4f} {c['accept']:>8.4f} "
              f"{c['open']:>8.4f} {c['exact_current']:>10.4f}")


if __name__ == "__main__":
    main()
