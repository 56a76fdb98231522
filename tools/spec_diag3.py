#!/usr/bin/env python3
"""Diagnostic: the speculative kernel's per-batch records (abvar/libmhgpu_specdbg.so,
MH_SPEC_DEBUG) against the sequential chain's proposals and decisions from the oracle."""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as graft  # noqa: E402

os.environ["MH_SPEC"] = "1"
mh, orc = graft.load_package(), graft.load_oracle()
lib = mh.load_library(str(ROOT / "abvar" / "libmhgpu_specdbg.so"))
mh.abi._lib = lib
lib.mh_debug_spec.argtypes = [C.POINTER(C.c_uint), C.c_int]
n, chain, steps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
room = mh.synthetic_room(n)
seed = 5150
buf = (C.c_uint * 65536)()
print("[diag] session", flush=True)
with mh.Session(room, 1, seed=seed, chain_offset=chain) as s:
    print("[diag] created", s.step_kernel(), flush=True)
    s.run(steps)
    s.current_costs()
    print("[diag] ran", flush=True)
cnt = lib.mh_debug_spec(buf, 65536)
print("[diag] records", cnt, flush=True)
np.save(os.environ.get("MH_DIAG_OUT", "/tmp/spec_records.npy"),
        np.frombuffer(bytes(buf), dtype=np.uint32)[:cnt])
d = np.frombuffer(bytes(buf), dtype=np.uint32)[:cnt]
f = lambda u: np.array([u], dtype=np.uint32).view(np.float32)[0]
# sequential proposals from the oracle's primitives
o = orc.load()
r = orc.rng_init(seed, chain)
sx = np.float32(room.surface_rectangle[0].x - room.surface_rectangle[2].x) / np.float32(16)
props = []
for t in range(steps + 16):
    mode = o.orc_rand_int(C.byref(r), 2, 0)
    k1 = k2 = -1
    d1 = d2 = np.float32(0)
    if mode == 0:
        k1 = o.orc_pick_object(C.cast(room.cfg, C.c_void_p), n, C.byref(r))
        d1 = np.float32(o.orc_rng_normal(C.byref(r))) * sx
        d2 = np.float32(o.orc_rng_normal(C.byref(r))) * sx
    elif mode == 1:
        k1 = o.orc_pick_object(C.cast(room.cfg, C.c_void_p), n, C.byref(r))
        d1 = np.float32(np.float64(np.float32(o.orc_rng_normal(C.byref(r)))) * (15.0 / 90.0 * 3.1416))
    elif n >= 2:
        k1 = o.orc_pick_object(C.cast(room.cfg, C.c_void_p), n, C.byref(r))
        k2 = o.orc_pick_object(C.cast(room.cfg, C.c_void_p), n, C.byref(r))
    u = np.float32(o.orc_rng_uniform(C.byref(r)))
    props.append((mode, k1, k2, float(d1), float(d2), float(u)))
acc = [int(orc.run_chains(room, 1, k, seed, chain_begin=chain)[2][0]) for k in range(0, steps + 1)]
accept = [acc[k + 1] - acc[k] for k in range(steps)]
rec = 7 + 8 * 8
for b in range(0, len(d), rec):
    done, kb, off, bmh, gs, com = [int(x) for x in d[b:b + 6]]
    gs = gs if gs < 2**31 else gs - 2**32
    print(f"batch done={done} kb={kb} off={off} bmh={bmh} gs={gs} committed={com} cur={f(d[b + 6]):.7g}")
    for g in range(8):
        q = d[b + 7 + 8 * g: b + 15 + 8 * g]
        mode, k1, k2, live = [int(x) if x < 2**31 else int(x) - 2**32 for x in q[:4]]
        dev = (mode, k1, k2, float(f(q[4])), float(f(q[5])), float(f(q[6])))
        t = done + g
        ok = t < len(props) and dev == props[t]
        print(f"   g{g} live={live} dev={dev} star={f(q[7]):.7g}" +
              ("" if ok or not live else f"  <-- oracle step {t}: {props[t] if t < len(props) else None}") +
              (f" oracle accepts={accept[t]}" if live and t < steps else ""))
