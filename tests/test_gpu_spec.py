"""The speculative step kernel (mh_spec.hip: rooms of at most 8 objects with few chains; a batch
evaluates the 8 or 16 nodes of a tree of accept / reject histories of one chain and commits the
realised path) against the oracle's sequential chain, bit for bit: every chain's final poses and
costs, over rooms whose acceptance rates grow different trees, for both instances (halves H = 1:
two wavefronts and 8 nodes per chain; H = 2: four wavefronts and 16 nodes, whose two chain
wavefronts keep the chain's state in step and commit a node of the other half by re-applying
the realised path)."""
import numpy as np
import pytest

from parity_util import check_chains

pytestmark = pytest.mark.gpu

PI = 3.1416


def _room(mh, kind, n):
    if kind == "frozen":
        return mh.synthetic_room(n, freeze_every=3)
    if kind == "manyrel":
        return mh.synthetic_room(n, n_rel=16 if n > 1 else None)
    room = mh.synthetic_room(n)
    if kind == "wrap":  # angle ranges crossing zero: the fmodf branch of Kernel.cu:245-250
        for k in range(room.srf.nRelationships):
            room.rsa[k].angleMin = 7 * PI / 4
            room.rsa[k].angleMax = PI / 4
    if kind in ("flat", "steep"):  # acceptance near 1 / low: the tree grows deep accept / reject
        scale = 0.0 if kind == "flat" else 40.0  # paths (spec_tree adapts every 32 batches)
        for w in ("WeightFocalPoint", "WeightPairWise", "WeightVisualBalance", "WeightSymmetry",
                  "WeightClearance", "WeightSurfaceArea"):
            setattr(room.srf, w, getattr(room.srf, w) * scale)
    if kind == "cramped":  # objects piled up: many Clearance / SurfaceArea terms, symmetry ties
        for j in range(n):
            room.cfg[j].x = 0.3 * (j % 3)
            room.cfg[j].y = 0.2 * (j // 3)
            room.cfg[j].rotY = 0.0
    return room


@pytest.mark.parametrize("halves", [1, 2])
@pytest.mark.parametrize("kind,n,chains,steps", [
    ("syn", 8, 1024, 2000),   # config 2's room and chain count
    ("syn", 8, 300, 2500),    # three launches: batches end at a launch's last step
    ("syn", 1, 64, 500),      # a single object: swaps draw nothing (Kernel.cu:657)
    ("syn", 2, 128, 800),
    ("syn", 5, 256, 700),
    ("frozen", 8, 256, 900),  # frozen picks are redrawn
    ("manyrel", 8, 128, 600),  # 16 relationships: two slots per lane
    ("wrap", 8, 128, 600),
    ("cramped", 8, 128, 600),
    ("frozen", 3, 64, 400),
    ("flat", 8, 128, 1500),   # every proposal accepted (u < 1): all-accept trees
    ("steep", 8, 128, 1500),  # few accepted: near-linear trees
    ("flat", 2, 64, 1200),
])
def test_spec_chains_match_oracle(mh, orc, hiplib, monkeypatch, halves, kind, n, chains, steps):
    monkeypatch.setenv("MH_SPEC", "1")
    monkeypatch.setenv("MH_SPEC_H", str(halves))
    room = _room(mh, kind, n)
    seed = 5150 + n + chains
    with mh.Session(room, chains, seed=seed) as s:
        assert s.step_kernel() == (128 * halves, 1, "speculative")  # (2H wavefronts per chain)
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
        cur = s.current_costs()
        acc = s.summary().accepted
    if kind == "flat":
        assert acc > 0.99 * chains * steps
    ref_pts, ref_costs, _ = orc.run_chains(room, chains, steps, seed, threads=8)
    check_chains(f"speculative H={halves} {kind} N={n}", pts, costs, ref_pts, ref_costs,
                 report=True)
    # the costs each chain carries equal the final pass's, OffLimits aside
    keep = [0, 1, 2, 3, 4, 5, 7]
    assert np.array_equal(cur[:, keep].view(np.uint32), costs[:, keep].view(np.uint32))


@pytest.mark.parametrize("halves", [1, 2])
def test_spec_resume_split_runs(mh, hiplib, monkeypatch, halves):
    """k runs of m steps equal one run of k m steps (the stream, the Box-Muller cache and the
    accepted count resume exactly across batch and launch boundaries)."""
    monkeypatch.setenv("MH_SPEC", "1")
    monkeypatch.setenv("MH_SPEC_H", str(halves))
    room = mh.synthetic_room(8)
    with mh.Session(room, 96, seed=77) as s:
        for m in (1, 2, 3, 7, 8, 9, 13, 999, 1000, 1001):
            s.run(m)
        s.finalize()
        p1, c1 = s.download()
        a1 = s.summary().accepted
    with mh.Session(room, 96, seed=77) as s:
        s.run(3043)
        s.finalize()
        p2, c2 = s.download()
        a2 = s.summary().accepted
    assert np.array_equal(p1.view(np.uint32), p2.view(np.uint32))
    assert np.array_equal(c1.view(np.uint32), c2.view(np.uint32))
    assert a1 == a2


def test_spec_is_the_default_for_few_small_chains(mh, hiplib, monkeypatch):
    """The plain family, rooms of at most 8 objects, at most 64 chains per CU (measured faster
    than the full-evaluation kernels there); MH_SPEC=0 opts out."""
    monkeypatch.delenv("MH_SPEC", raising=False)
    monkeypatch.delenv("MH_SPEC_H", raising=False)
    monkeypatch.delenv("MH_DELTA", raising=False)
    monkeypatch.delenv("MH_SPEC_BOUND", raising=False)
    cus = mh.device_cus()
    with mh.Session(mh.synthetic_room(8), 1024, seed=1) as s:
        assert s.step_kernel()[2] == "speculative"
    # the 16-node instance up to two chains per CU, the 8-node one beyond (config 2's 1,024
    # chains on 256 CUs)
    # chains per CU; the instance deciding on the bound (two wavefronts per SIMD) up to four
    # chains per CU (config 2), the exact one (98 VGPRs; LDS-bound residency) beyond
    with mh.Session(mh.synthetic_room(8), 2 * cus, seed=1) as s:
        assert s.step_kernel() == (256, 1, "speculative") and s.occupancy() == 2
    with mh.Session(mh.synthetic_room(8), 2 * cus + 1, seed=1) as s:
        assert s.step_kernel() == (128, 1, "speculative") and s.occupancy() == 4
    with mh.Session(mh.synthetic_room(8), 4 * cus + 1, seed=1) as s:
        assert s.step_kernel() == (128, 1, "speculative") and s.occupancy() >= 5
    monkeypatch.setenv("MH_SPEC_BOUND", "0")
    with mh.Session(mh.synthetic_room(8), 2 * cus, seed=1) as s:
        assert s.step_kernel() == (256, 1, "speculative") and s.occupancy() == 4
    monkeypatch.delenv("MH_SPEC_BOUND")
    with mh.Session(mh.synthetic_room(8), 1024, seed=1, track=1) as s:  # (plain family only)
        assert s.step_kernel()[2] != "speculative"
    with mh.Session(mh.synthetic_room(16), 1024, seed=1) as s:
        assert s.step_kernel()[2] != "speculative"
    # the cutoff is 64 chains per CU of this device (16,384 on MI355X's 256 CUs; another SKU or
    # a compute-partition mode moves it)
    cut = 64 * cus
    with mh.Session(mh.synthetic_room(8), cut, seed=1) as s:
        assert s.step_kernel()[2] == "speculative"
    with mh.Session(mh.synthetic_room(8), cut + 1, seed=1) as s:
        assert s.step_kernel()[2] != "speculative"
    with mh.Session(mh.synthetic_room(8), max(1 << 16, 2 * cut), seed=1) as s:  # fills the GPU
        assert s.step_kernel()[2] != "speculative"
    monkeypatch.setenv("MH_SPEC", "0")
    with mh.Session(mh.synthetic_room(8), 1024, seed=1) as s:
        assert s.step_kernel()[2] != "speculative"
