#!/usr/bin/env python3
"""Regenerates tests/golden/golden.json: the fixtures every parity test is anchored to.

* kat_main_fixture: the reference's own Costs() on its main() room (Kernel.cu:1007-1166), as
  recorded in SURVEY.md 8(c) -- data, not generated here.
* rng: the first draws of a few (seed, subsequence) Philox streams (oracle restatement, which is
  itself pinned to the Random123 KAT vectors in tests/test_oracle.py).
* chains: hashes of the oracle's final poses/costs for seeded runs of the defined chain on the
  main() room and synthetic rooms; the HIP path must reproduce them bit for bit.
* rooms: hashes of the synthetic rooms' wire bytes (SURVEY.md 8(d) generator).
* xorwow_rocrand: the first draws of rocRAND's own XORWOW engine (xorwow_rocrand.cpp, built here
  with hipcc for the host) -- pins the oracle's XORWOW recurrence and subsequence jump.
* index_n: chains whose pick draws u == 1.0f early (written by find_index_n.py; kept here).
* xorwow_curand / chains_xorwow: the oracle's cuRAND-XORWOW streams and seeded chain runs in
  that mode (the HIP path must reproduce them bit for bit).

Run from the repo root:  python tests/golden/make_golden.py
"""
import ctypes as C
import hashlib
import json
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as graft  # noqa: E402

CHAIN_CASES = [
    {"room": "main_fixture", "n": 32, "chains": 64, "steps": 40, "seed": 20251015},
    {"room": "synthetic", "n": 8, "chains": 256, "steps": 300, "seed": 7},
    {"room": "synthetic", "n": 64, "chains": 16, "steps": 100, "seed": 42},
    {"room": "synthetic", "n": 256, "chains": 4, "steps": 20, "seed": 5},
    {"room": "synthetic_frozen", "n": 16, "chains": 64, "steps": 200, "seed": 11},
]
RNG_CASES = [(42, 0), (42, 65535), (2**63 + 5, 123456789)]
XORWOW_CASES = [(1760000000, 0), (1760000000 + 4097, 4097), (7, 2**40 + 3)]
XORWOW_CHAIN_CASES = [
    {"room": "main_fixture", "n": 32, "chains": 64, "steps": 40, "seed": 1760000000},
    {"room": "synthetic", "n": 64, "chains": 16, "steps": 100, "seed": 42},
]


def rocrand_xorwow_vectors():
    src = Path(__file__).with_name("xorwow_rocrand.cpp")
    with tempfile.TemporaryDirectory() as d:
        exe = Path(d) / "xorwow_rocrand"
        subprocess.run(["/opt/rocm/bin/hipcc", "-O1", str(src), "-o", str(exe)], check=True)
        return json.loads(subprocess.run([str(exe)], check=True, capture_output=True,
                                         text=True).stdout)


def make_room(mh, case):
    if case["room"] == "main_fixture":
        return mh.main_fixture()
    if case["room"] == "synthetic_frozen":
        return mh.synthetic_room(case["n"], freeze_every=4)
    return mh.synthetic_room(case["n"])


def sha(a) -> str:
    return hashlib.sha256(bytes(memoryview(a))).hexdigest()


def room_bytes(room) -> bytes:
    parts = [room.srf, room.cfg, room.rss, room.rsa, room.clearances, room.offlimits,
             room.vertices, room.surface_rectangle]
    return b"".join(bytes(memoryview(p)) if not isinstance(p, C.Structure) else bytes(p)
                    for p in parts)


def main():
    mh, orc = graft.load_package(), graft.load_oracle()
    out = {"kat_main_fixture": {
        "totalCosts": 3921.14038, "PairWiseCosts": 0.0, "VisualBalanceCosts": -65.7609329,
        "FocalPointCosts": 36.7696877, "SymmetryCosts": 46.1316452, "ClearanceCosts": 16.0,
        "OffLimitsCosts": 0.0, "SurfaceAreaCosts": 3888.0,
        "source": "SURVEY.md 8(c): reference Costs() on Kernel.cu:1007-1166, WeightOffLimits=0"}}
    out["rng"] = []
    for seed, sub in RNG_CASES:
        u, f, g = orc.rng_streams(seed, sub, 16)
        out["rng"].append({"seed": seed, "subsequence": sub, "u32": [int(x) for x in u],
                           "uniform_bits": [int(x) for x in f.view("uint32")],
                           "normal_bits": [int(x) for x in g.view("uint32")]})
    out["chains"] = []
    for case in CHAIN_CASES:
        room = make_room(mh, case)
        pts, costs, acc = orc.run_chains(room, case["chains"], case["steps"], case["seed"],
                                         threads=8)
        out["chains"].append(dict(case, points_sha256=sha(pts), costs_sha256=sha(costs),
                                  mean_total=float(costs[:, 0].astype("float64").mean()),
                                  accepted=int(acc.sum())))
    out["xorwow_rocrand"] = rocrand_xorwow_vectors()
    out["xorwow_curand"] = []
    for seed, sub in XORWOW_CASES:
        u, f, g = orc.rng_streams(seed, sub, 16, kind=orc.XORWOW_CURAND)
        out["xorwow_curand"].append({"seed": seed, "subsequence": sub, "u32": [int(x) for x in u],
                                     "uniform_bits": [int(x) for x in f.view("uint32")],
                                     "normal_bits": [int(x) for x in g.view("uint32")]})
    out["chains_xorwow"] = []
    for case in XORWOW_CHAIN_CASES:
        room = make_room(mh, case)
        st, costs, acc = orc.run_chains(room, case["chains"], case["steps"], case["seed"],
                                        threads=8, rng=1)
        pts = st.astype("float32")
        out["chains_xorwow"].append(dict(case, points_sha256=sha(pts), costs_sha256=sha(costs),
                                         mean_total=float(costs[:, 0].astype("float64").mean()),
                                         accepted=int(acc.sum())))
    out["rooms"] = {f"synthetic{n}": hashlib.sha256(room_bytes(mh.synthetic_room(n))).hexdigest()
                    for n in (1, 8, 64, 256)}
    path = Path(__file__).with_name("golden.json")
    if path.exists():  # searched fixtures (find_index_n.py, find_u1_accept.py) are kept
        old = json.loads(path.read_text())
        out["index_n"] = old.get("index_n", [])
        out["u1_accept"] = old.get("u1_accept", [])
    path.write_text(json.dumps(out, indent=1) + "\n")
    print("wrote", path)


if __name__ == "__main__":
    main()
