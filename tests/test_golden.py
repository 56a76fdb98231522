"""Committed fixtures (tests/golden/golden.json, made by tests/golden/make_golden.py): the oracle
and the room generator must keep reproducing them (CPU); the HIP path must reproduce the chain
fixtures bit for bit (GPU, in test_gpu_parity.py)."""
import hashlib
import importlib.util
import json
from pathlib import Path

import numpy as np
import pytest

GOLDEN = json.loads((Path(__file__).parent / "golden" / "golden.json").read_text())
_spec = importlib.util.spec_from_file_location(
    "make_golden", Path(__file__).parent / "golden" / "make_golden.py")
make_golden = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(make_golden)


def test_golden_kat_is_the_oracle_answer(mh, orc):
    got = orc.costs(mh.main_fixture())
    kat = GOLDEN["kat_main_fixture"]
    for k, name in enumerate(mh.COST_FIELDS):
        assert got[k] == pytest.approx(kat[name], rel=1e-8, abs=1e-12)


@pytest.mark.parametrize("case", GOLDEN["rng"], ids=lambda c: f"{c['seed']}-{c['subsequence']}")
def test_golden_rng(orc, case):
    u, f, g = orc.rng_streams(case["seed"], case["subsequence"], 16)
    assert [int(x) for x in u] == case["u32"]
    assert [int(x) for x in f.view(np.uint32)] == case["uniform_bits"]
    assert [int(x) for x in g.view(np.uint32)] == case["normal_bits"]


@pytest.mark.parametrize("case", GOLDEN["chains"], ids=lambda c: f"{c['room']}{c['n']}")
def test_golden_chains_oracle(mh, orc, case):
    room = make_golden.make_room(mh, case)
    pts, costs, acc = orc.run_chains(room, case["chains"], case["steps"], case["seed"], threads=8)
    assert make_golden.sha(pts) == case["points_sha256"]
    assert make_golden.sha(costs) == case["costs_sha256"]
    assert int(acc.sum()) == case["accepted"]


@pytest.mark.parametrize("n", [1, 8, 64, 256])
def test_golden_rooms(mh, n):
    room = mh.synthetic_room(n)
    h = hashlib.sha256(make_golden.room_bytes(room)).hexdigest()
    assert h == GOLDEN["rooms"][f"synthetic{n}"]
    assert room.srf.nClearances == n // 4 and room.srf.nRelationships == (n // 2 if n > 1 else 0)
    w = room.surface_rectangle[0].x
    base = np.ctypeslib.as_array(room.cfg)
    assert np.all((base["x"] >= 0) & (base["x"] <= w) & (base["y"] >= 0) & (base["y"] <= w))


@pytest.mark.parametrize("case", GOLDEN["xorwow_rocrand"],
                         ids=lambda c: f"{c['seed']}-{c['subsequence']}")
def test_oracle_xorwow_matches_rocrand_engine(orc, case):
    """The oracle's XORWOW (its own GF(2) subsequence jump) run with rocRAND's seeding constants
    reproduces rocRAND's xorwow_engine (tests/golden/xorwow_rocrand.cpp): the recurrence, the
    Weyl sequence and the 2^67-draw jump it shares with cuRAND are pinned; only the seeding
    constants differ between the two libraries."""
    u, _, _ = orc.rng_streams(case["seed"], case["subsequence"], 8, kind=orc.XORWOW_ROCRAND)
    assert [int(x) for x in u] == case["u32"]


@pytest.mark.parametrize("case", GOLDEN["xorwow_curand"],
                         ids=lambda c: f"{c['seed']}-{c['subsequence']}")
def test_golden_xorwow_curand(orc, case):
    u, f, g = orc.rng_streams(case["seed"], case["subsequence"], 16, kind=orc.XORWOW_CURAND)
    assert [int(x) for x in u] == case["u32"]
    assert [int(x) for x in f.view(np.uint32)] == case["uniform_bits"]
    assert [int(x) for x in g.view(np.uint32)] == case["normal_bits"]


@pytest.mark.parametrize("case", GOLDEN["chains_xorwow"], ids=lambda c: f"{c['room']}{c['n']}")
def test_golden_chains_xorwow_oracle(mh, orc, case):
    room = make_golden.make_room(mh, case)
    st, costs, acc = orc.run_chains(room, case["chains"], case["steps"], case["seed"], threads=8,
                                    rng=1)
    assert make_golden.sha(st.astype(np.float32)) == case["points_sha256"]
    assert make_golden.sha(costs) == case["costs_sha256"]
    assert int(acc.sum()) == case["accepted"]


@pytest.mark.parametrize("case", GOLDEN["index_n"], ids=lambda c: f"chain{c['chain']}")
def test_index_n_fixture_reaches_the_edge(mh, orc, case):
    """The searched chains (find_index_n.py) draw index nObjs (u == 1.0f, Kernel.cu:566-574)
    at step `first_step` and not before; the defined semantics redraw it."""
    room = mh.synthetic_room(case["n"])
    orc.index_n_draws(reset=True)
    orc.run_chains(room, 1, case["first_step"] - 1, case["seed"], chain_begin=case["chain"])
    assert orc.index_n_draws() == 0
    orc.index_n_draws(reset=True)
    _, costs, _ = orc.run_chains(room, 1, case["steps"], case["seed"], chain_begin=case["chain"])
    assert orc.index_n_draws() >= 1
    assert np.isfinite(costs).all()
