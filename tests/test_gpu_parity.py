"""Parity of the HIP path (libmhgpu.so through its C ABI) with the oracle (oracle/mh_oracle.c,
the C restatement of KernelFolder/Kernel/Kernel.cu:162-828).

Bar: the RNG streams, the cost components and every chain's final points and costs are compared
BIT FOR BIT; a single forked chain fails the test, and the failure names its global id
(tests/parity_util.py). The mean final total is also checked against the north-star tolerance
(1e-4 relative). Config-length runs are in tests/test_gpu_configs.py.
"""
import ctypes as C

import numpy as np
import pytest

from parity_util import check_chains

pytestmark = pytest.mark.gpu

PI = 3.1416


def _room(mh, kind: str, n: int):
    if kind == "main":
        return mh.main_fixture()
    if kind == "frozen":
        return mh.synthetic_room(n, freeze_every=4)
    if kind == "manyrel":  # more relationships than objects: R > N + 1
        return mh.synthetic_room(n, n_rel=3 * n + 5)
    room = mh.synthetic_room(n)
    if kind == "wrap":  # angle ranges crossing zero: the fmodf branch of Kernel.cu:245-250
        for k in range(room.srf.nRelationships):
            room.rsa[k].angleMin = 7 * PI / 4
            room.rsa[k].angleMax = PI / 4
    return room


def _narrow_lanes(n: int) -> int:
    """The narrowest full-evaluation width for N objects (next power of two >= N, 8..64): the
    library widens chains when they are few (choose_lanes), so the tests pin the narrow
    instances (several chains per wavefront) explicitly."""
    L = 8
    while L < n and L < 64:
        L *= 2
    return L


STEPS = ["incremental", "full", "full-narrow", "full-capped"]


def _use_step(monkeypatch, step: str, n: int) -> str:
    """Selects the step kernel (MH_DELTA) and, for "full-narrow", the narrow width (MH_LANES);
    "full-capped" forces the register-capped instance of the one-chain-per-wavefront step that
    launches of many chains use (these tests' few chains get the uncapped OP_STEP_FEW one).
    Returns the step-kernel kind the session must report."""
    kind = step.split("-")[0]
    monkeypatch.setenv("MH_DELTA", "1" if kind == "incremental" else "0")
    monkeypatch.setenv("MH_SPEC", "0")  # (tests/test_gpu_spec.py covers the speculative kernel)
    if step == "full-narrow":
        if _narrow_lanes(n) == 64:
            pytest.skip("the narrow instance is the default one for this N")
        monkeypatch.setenv("MH_LANES", str(_narrow_lanes(n)))
    if step == "full-capped":
        if n > 64:
            pytest.skip("one object per lane only")
        monkeypatch.setenv("MH_STEP_FEW", "0")
    return kind


def _random_cfgs(mh, room, k: int, seed: int):
    """k configurations of room.n objects: uniform poses plus out-of-room objects, rotY at 0,
    2*PI and just inside, swapped duplicates, and coincident objects."""
    rng = np.random.default_rng(seed)
    n = room.n
    xs = [room.surface_rectangle[i].x for i in range(4)]
    w = max(xs) - min(xs)
    base = np.ctypeslib.as_array(room.cfg)
    arr = (mh.abi.positionAndRotation * (k * n))()
    for c in range(k):
        for i in range(n):
            b = base[i]
            x = rng.uniform(-0.25 * w, 1.25 * w) if (c % 3 == 0) else rng.uniform(0, w)
            y = rng.uniform(-0.25 * w, 1.25 * w) if (c % 3 == 0) else rng.uniform(0, w)
            rot = [0.0, 2 * PI, 1e-7, 2 * PI - 1e-7, rng.uniform(0, 2 * PI)][(c + i) % 5]
            if c % 7 == 3 and i > 0:  # coincident with object 0
                x, y = arr[c * n].x, arr[c * n].y
            arr[c * n + i] = mh.abi.positionAndRotation(
                x, y, rng.uniform(-1, 1), rng.uniform(-1, 1), rot, rng.uniform(-1, 1),
                bool(b["frozen"]), float(b["length"]), float(b["width"]))
    return arr


def _oracle_costs(orc, room, cfgs, k):
    n = room.n
    out = np.zeros((k, 8), dtype=np.float32)
    size = C.sizeof(cfgs._type_)
    for c in range(k):
        sub = (cfgs._type_ * n).from_address(C.addressof(cfgs) + c * n * size)
        out[c] = orc.costs(room, sub)
    return out


def _report_match(name, got, ref):
    same = np.all(got.view(np.uint32) == ref.view(np.uint32), axis=tuple(range(1, got.ndim)))
    denom = np.maximum(np.abs(ref), 1e-6)
    rel = np.abs(got.astype(np.float64) - ref) / denom
    print(f"{name}: {same.mean() * 100:.2f}% bit-identical, max rel diff {rel.max():.3g}")
    return same, rel


def test_rng_streams_match(mh, orc, hiplib):
    for seed, sub in [(0, 0), (42, 7), (2**63 + 5, 123456789), (0xDEADBEEF, 65535)]:
        u, f, g = mh.debug_rng(seed, sub, 4099)
        ru, rf, rg = orc.rng_streams(seed, sub, 4099)
        assert np.array_equal(u, ru), "Philox words differ"
        assert np.array_equal(f.view(np.uint32), rf.view(np.uint32)), "uniforms differ"
        bad = np.flatnonzero(g.view(np.uint32) != rg.view(np.uint32))
        assert bad.size == 0, f"normals differ at draws {bad[:16].tolist()}"
        assert f.min() > 0.0 and f.max() <= 1.0


def test_costs_main_fixture_known_answer(mh, orc, hiplib):
    room = mh.main_fixture()
    got = mh.evaluate_costs(room, room.cfg)[0]
    kat = np.array([3921.14038, 0, -65.7609329, 36.7696877, 46.1316452, 16, 0, 3888],
                   dtype=np.float32)  # the reference's own Costs()
    assert np.allclose(got, kat, rtol=1e-8, atol=0)
    assert np.array_equal(got.view(np.uint32), orc.costs(room).view(np.uint32))


@pytest.mark.parametrize("kind,n", [("main", 32), ("syn", 1), ("syn", 2), ("syn", 5),
                                    ("syn", 8), ("frozen", 16), ("wrap", 31), ("syn", 32),
                                    ("syn", 50), ("syn", 64), ("wrap", 64), ("syn", 100),
                                    ("syn", 256)])
def test_costs_match_oracle(mh, orc, hiplib, kind, n):
    room = _room(mh, kind, n)
    k = 48 if n <= 64 else 12
    cfgs = _random_cfgs(mh, room, k, seed=n * 7 + len(kind))
    got = mh.evaluate_costs(room, cfgs)
    ref = _oracle_costs(orc, room, cfgs, k)
    same, rel = _report_match(f"costs {kind} N={room.n}", got, ref)
    bad = np.flatnonzero(~same)
    assert bad.size == 0, (f"costs {kind} N={room.n}: configurations {bad.tolist()} differ "
                           f"(max rel {rel.max():.3g})")


@pytest.mark.parametrize("kind,n,chains,steps", [
    ("main", 32, 256, 100),      # config 1's room (Kernel.cu:1007-1194)
    ("syn", 8, 1024, 300),       # config 2's room
    ("frozen", 16, 128, 200),    # frozen objects: redraw loop
    ("wrap", 24, 128, 150),
    ("syn", 5, 64, 200),
    ("syn", 1, 32, 50),          # swap with nObjs < 2 draws nothing more (Kernel.cu:657)
    ("syn", 64, 64, 150),        # config 3's room
    ("syn", 64, 192, 1500),      # long chains: the cached symmetry row maxima over many accepts
    ("syn", 20, 512, 2000),      # L = 32, two chains per wave
    ("syn", 100, 16, 60),        # NPL = 2
    ("syn", 256, 8, 25),         # config 5's room
])
@pytest.mark.parametrize("geometry", ["default", "narrow"])
def test_chains_match_oracle(mh, orc, hiplib, monkeypatch, geometry, kind, n, chains, steps):
    if geometry == "narrow":
        if _narrow_lanes(n) == 64:
            pytest.skip("the narrow instance is the default one for this N")
        monkeypatch.setenv("MH_LANES", str(_narrow_lanes(n)))
    room = _room(mh, kind, n)
    seed = 1000 + n
    pts, costs = mh.kernel_wrapper(room, chains, steps, seed=seed)
    ref_pts, ref_costs, _ = orc.run_chains(room, chains, steps, seed, threads=8)
    check_chains(f"{kind} N={n} {chains}x{steps}", pts, costs, ref_pts, ref_costs)


@pytest.mark.parametrize("step", STEPS)
@pytest.mark.parametrize("kind,n,chains,steps", [
    ("main", 32, 128, 300),
    ("frozen", 16, 128, 400),
    ("wrap", 24, 96, 400),
    ("syn", 2, 64, 300),
    ("syn", 9, 128, 500),
    ("syn", 64, 64, 600),
    ("syn", 100, 16, 120),
    ("manyrel", 8, 64, 300),
    ("manyrel", 100, 16, 100),
])
def test_chains_match_oracle_each_step_kernel(mh, orc, hiplib, monkeypatch, step, kind, n,
                                              chains, steps):
    """Both step kernels (MH_DELTA=1: incremental evaluation, mh_delta.hip; MH_DELTA=0: full
    evaluation, mh_chain.hip) against the oracle, whichever is the default for N."""
    kind_ = _use_step(monkeypatch, step, n)
    room = _room(mh, kind, n)
    seed = 7000 + n
    with mh.Session(room, chains, seed=seed) as s:
        assert s.step_kernel()[2].split("-")[0] == kind_
        if step in ("full", "full-capped") and n <= 64:  # (which one-object-per-lane instance)
            assert s.step_kernel()[2] == ("full-few" if step == "full" else "full")
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
    ref_pts, ref_costs, _ = orc.run_chains(room, chains, steps, seed, threads=8)
    check_chains(f"{step} {kind} N={n}", pts, costs, ref_pts, ref_costs)


def test_chains_over_launch_chunks(mh, orc, hiplib):
    """1200 steps span two launches (1000 steps per launch): resumption is exact."""
    room = mh.synthetic_room(8)
    pts, costs = mh.kernel_wrapper(room, 32, 1200, seed=99)
    ref_pts, ref_costs, _ = orc.run_chains(room, 32, 1200, 99, threads=8)
    check_chains("N=8 1200 steps", pts, costs, ref_pts, ref_costs)


def test_session_resume_and_offsets(mh, hiplib):
    room = mh.synthetic_room(16)
    with mh.Session(room, 100, seed=7) as s:
        s.run(60)
        s.finalize()
        p1, c1 = s.download()
        summ = s.summary()
    with mh.Session(room, 100, seed=7) as s:
        s.run(25)
        s.run(0)
        s.run(35)
        s.finalize()
        p2, c2 = s.download()
    assert np.array_equal(p1, p2) and np.array_equal(c1, c2)
    with mh.Session(room, 40, seed=7, chain_offset=60) as s:  # a rank's shard
        s.run(60)
        s.finalize()
        p3, c3 = s.download()
        summ3 = s.summary()
    assert np.array_equal(p3, p1[60:]) and np.array_equal(c3, c1[60:])
    assert summ.n_chains == 100 and summ3.n_chains == 40
    assert summ.best_total == c1[:, 0].max()
    assert summ.best_chain == int(np.argmax(c1[:, 0]))
    assert summ3.best_chain == 60 + int(np.argmax(c3[:, 0]))
    assert abs(summ.sum_total - c1[:, 0].astype(np.float64).sum()) <= 1e-6 * abs(summ.sum_total)


def test_seed_determinism_and_independence(mh, hiplib):
    room = mh.synthetic_room(12)
    a = mh.kernel_wrapper(room, 64, 80, seed=5)
    b = mh.kernel_wrapper(room, 64, 80, seed=5)
    c = mh.kernel_wrapper(room, 64, 80, seed=6)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert not np.array_equal(a[0], c[0])
    # distinct chains draw distinct streams
    assert len({a[0][i].tobytes() for i in range(64)}) == 64


def test_zero_iterations_returns_input_pose(mh, orc, hiplib):
    room = mh.synthetic_room(9)
    pts, costs = mh.kernel_wrapper(room, 4, 0, seed=1)
    base = np.ctypeslib.as_array(room.cfg)
    for k, f in enumerate(["x", "y", "z", "rotX", "rotY", "rotZ"]):
        assert np.array_equal(pts[:, :, k], np.broadcast_to(base[f].astype(np.float32), (4, 9)))
    assert np.array_equal(costs[0].view(np.uint32), orc.costs(room).view(np.uint32))


def test_full_size_config3_properties(mh, orc, hiplib):
    """Config 3's shape (N=64, 65,536 chains) at 20 steps: properties that hold at any size,
    plus chains sampled across the range checked against the oracle by global id."""
    room = mh.synthetic_room(64)
    chains, steps, seed = 65536, 20, 42
    with mh.Session(room, chains, seed=seed) as s:
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
        summ = s.summary()
    w = room.surface_rectangle[0].x
    assert np.all((pts[:, :, 0] >= 0) & (pts[:, :, 0] <= np.float32(w)))
    assert np.all((pts[:, :, 1] >= 0) & (pts[:, :, 1] <= np.float32(w)))
    assert summ.n_chains == chains
    assert summ.best_total == costs[:, 0].max()
    assert 0 < summ.accepted <= chains * steps
    for cid in [0, 1, 4097, 32768, 65535]:
        rp, rc, _ = orc.run_chains(room, 1, steps, seed, chain_begin=cid)
        assert np.array_equal(pts[cid].view(np.uint32), rp[0].view(np.uint32)), cid
        assert np.array_equal(costs[cid].view(np.uint32), rc[0].view(np.uint32)), cid


RUNNING_CASES = [(n, ch, st, step) for n, ch, st in [(64, 65536, 400), (20, 16384, 1500),
                                                      (256, 8192, 200), (5, 4096, 3000)]
                 for step in ("incremental", "full")] + [(5, 4096, 3000, "speculative"),
                                                         (8, 16384, 2000, "speculative")]


@pytest.mark.parametrize("n,chains,steps,step", RUNNING_CASES)
def test_running_costs_equal_fresh_evaluation(mh, hiplib, monkeypatch, step, n, chains, steps):
    """Size-independent property of the incremental evaluation: after many accepted proposals,
    the costs every chain carries for its current state (symmetry row maxima updated
    incrementally; the speculative kernel's adopted node's costs) equal a full re-evaluation of
    that state, bit for bit, on every chain."""
    monkeypatch.setenv("MH_DELTA", "1" if step == "incremental" else "0")
    monkeypatch.setenv("MH_SPEC", "1" if step == "speculative" else "0")
    room = mh.synthetic_room(n)
    with mh.Session(room, chains, seed=77 + n) as s:
        assert s.step_kernel()[2].split("-")[0] == step
        s.run(steps)
        s.finalize()
        _, fresh = s.download()
        running = s.current_costs()
        acc = s.summary().accepted
    assert acc > chains * steps // 20
    keep = [0, 1, 2, 3, 4, 5, 7]  # all but OffLimits, which the step path does not evaluate
    same = np.all(running[:, keep].view(np.uint32) == fresh[:, keep].view(np.uint32), axis=1)
    assert same.all(), f"{(~same).sum()} of {chains} chains drifted"
    assert np.all(running[:, 6] == 0)


def _golden():
    import importlib.util
    import json
    from pathlib import Path
    d = Path(__file__).parent / "golden"
    spec = importlib.util.spec_from_file_location("make_golden", d / "make_golden.py")
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return json.loads((d / "golden.json").read_text()), mg


GOLDEN, MAKE_GOLDEN = _golden()


@pytest.mark.parametrize("case", GOLDEN["chains"], ids=lambda c: f"{c['room']}{c['n']}")
def test_golden_chains_hip(mh, hiplib, case):
    room = MAKE_GOLDEN.make_room(mh, case)
    pts, costs = mh.kernel_wrapper(room, case["chains"], case["steps"], seed=case["seed"])
    assert MAKE_GOLDEN.sha(pts) == case["points_sha256"]
    assert MAKE_GOLDEN.sha(costs) == case["costs_sha256"]


@pytest.mark.parametrize("case", GOLDEN["rng"], ids=lambda c: f"{c['seed']}-{c['subsequence']}")
def test_golden_rng_hip(mh, hiplib, case):
    u, f, g = mh.debug_rng(case["seed"], case["subsequence"], 16)
    assert [int(x) for x in u] == case["u32"]
    assert [int(x) for x in f.view(np.uint32)] == case["uniform_bits"]
    assert [int(x) for x in g.view(np.uint32)] == case["normal_bits"]


@pytest.mark.parametrize("L", [8, 16, 32, 64])
def test_group_collectives(mh, hiplib, L):
    """DPP / permlane group reductions and scans against numpy, with ties and negative values."""
    rng = np.random.default_rng(L)
    for trial in range(6):
        v = rng.normal(size=64).astype(np.float32)
        if trial % 2:
            v = np.round(v * 2) / 2  # many exact ties
        iv = rng.integers(-5, 9, size=64).astype(np.int32)
        got = mh.debug_collectives(L, v, iv)
        for g in range(64 // L):
            sl = slice(g * L, (g + 1) * L)
            vg, ig = v[sl], iv[sl]
            srt = np.sort(vg)[::-1]
            j = int(np.flatnonzero(vg == srt[0])[0])
            assert np.all(got["m1"][sl] == srt[0]) and np.all(got["m2"][sl] == srt[1])
            assert np.all(got["j1"][sl] == j) and np.all(got["arg"][sl] == j)
            assert np.all(got["max"][sl] == srt[0])
            assert np.array_equal(got["scan"][sl], np.concatenate([[0], np.cumsum(ig)[:-1]]))
            assert np.all(got["total"][sl] == ig.sum())
            assert np.all(got["imax"][sl] == ig.max()) and np.all(got["isum"][sl] == ig.sum())
        # wave_fsum8 (the rejection bound's eight wavefront sums, mh_common.h): exact integer
        # sums, the same value on every lane
        for k in range(8):
            want = sum(int(iv[(3 * lane + k) & 63]) + k for lane in range(64))
            assert np.all(got["wsum8"][k] == np.float32(want)), (k, got["wsum8"][k], want)


@pytest.mark.parametrize("step", STEPS)
@pytest.mark.parametrize("track", [1, 2])
@pytest.mark.parametrize("kind,n,chains,steps", [
    ("main", 32, 96, 300),
    ("frozen", 16, 128, 400),
    ("syn", 9, 128, 400),
    ("syn", 64, 48, 1200),   # two launches: the best total is carried in the chain meta
    ("syn", 2, 64, 200),
])
def test_best_of_chain_matches_oracle(mh, orc, hiplib, monkeypatch, step, track, kind, n, chains,
                                      steps):
    """Best-of-chain tracking (KernelWrapperEx / mh_session_create_ex; the reference's
    commented-out cfgBest, Kernel.cu:779-782,808-816,840-860) against the oracle's restatement:
    the best configuration and its eight costs, bit for bit, for both step kernels."""
    kind_ = _use_step(monkeypatch, step, n)
    room = _room(mh, kind, n)
    seed = 9100 + n + track
    with mh.Session(room, chains, seed=seed, track=track) as s:
        assert s.step_kernel()[2] == kind_  # (never the few-chains instance)
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
    ref_state, ref_costs, _ = orc.run_chains(room, chains, steps, seed, threads=8, track=track)
    check_chains(f"best({track}) {step} {kind} N={n}", pts, costs, ref_state, ref_costs)
    # the best is at least as good as the final current state of the same trajectory
    _, cur_costs = mh.kernel_wrapper(room, chains, steps, seed=seed)
    if track == 1:
        assert np.all(costs[:, 0] <= cur_costs[:, 0])
    else:
        assert np.all(costs[:, 0] >= cur_costs[:, 0])


def test_best_of_chain_kernel_wrapper_ex(mh, orc, hiplib):
    """KernelWrapperEx returns the best configurations in the reference's result layout, and
    track_best = OFF through it equals KernelWrapperSeeded."""
    room = mh.synthetic_room(64)
    chains, steps, seed = 256, 500, 77
    p_best, c_best = mh.kernel_wrapper(room, chains, steps, seed=seed, track=2)
    ref_state, ref_costs, _ = orc.run_chains(room, chains, steps, seed, threads=8, track=2)
    assert np.array_equal(p_best.view(np.uint32), ref_state.astype(np.float32).view(np.uint32))
    assert np.array_equal(c_best.view(np.uint32), ref_costs.view(np.uint32))
    p0, c0 = mh.kernel_wrapper(room, chains, steps, seed=seed)
    lib = mh.load_library()
    g = mh.abi.gpuConfig(chains, 0, 64, 0, 0, steps)
    res = lib.KernelWrapperEx(*room.args(), C.byref(g), C.byref(mh.abi.options(seed)))
    assert res
    try:
        pts = (mh.abi.point * (chains * room.n)).from_address(C.cast(res[0].points, C.c_void_p).value)
        p1 = np.frombuffer(bytes(memoryview(pts)), dtype=np.float32).reshape(chains, room.n, 6)
    finally:
        lib.KernelFreeResult(res)
    assert np.array_equal(p0.view(np.uint32), p1.view(np.uint32))


def test_best_of_chain_full_size(mh, hiplib):
    """Config 3's shape (65,536 chains, N = 64) with tracking on: the reported best costs equal
    a fresh evaluation of the reported best configurations (sampled), and best >= final."""
    room = mh.synthetic_room(64)
    chains, steps, seed = 65536, 300, 4242
    with mh.Session(room, chains, seed=seed, track=2) as s:
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
        summ = s.summary()
    with mh.Session(room, chains, seed=seed) as s0:
        s0.run(steps)
        s0.finalize()
        _, cur = s0.download()
    assert np.all(costs[:, 0] >= cur[:, 0])
    assert summ.best_total == costs[:, 0].max()
    idx = np.random.default_rng(0).choice(chains, 64, replace=False)
    cfgs = (mh.abi.positionAndRotation * (len(idx) * room.n))()
    base = np.ctypeslib.as_array(room.cfg)
    for j, c in enumerate(idx):
        for i in range(room.n):
            p = pts[c, i]
            cfgs[j * room.n + i] = mh.abi.positionAndRotation(
                *map(float, p), bool(base[i]["frozen"]), float(base[i]["length"]),
                float(base[i]["width"]))
    # the float points are a rounding of the double state, so compare totals loosely here;
    # the bit-exact check is test_best_of_chain_matches_oracle
    fresh = mh.evaluate_costs(room, cfgs)
    rel = np.abs(fresh[:, 0] - costs[idx, 0]) / np.maximum(np.abs(costs[idx, 0]), 1)
    assert np.median(rel) < 1e-3


# ---- cuRAND-XORWOW mode (mh_options.rng = MH_RNG_CURAND_XORWOW) ------------------------------

@pytest.mark.parametrize("case", GOLDEN["xorwow_curand"],
                         ids=lambda c: f"{c['seed']}-{c['subsequence']}")
def test_xorwow_streams_hip(mh, hiplib, case):
    """Device curand()/curand_uniform()/curand_normal() streams of curand_init(seed, sub, 0)
    (rocRAND's subsequence jump under cuRAND's seeding) equal the oracle's restatement (its own
    GF(2) jump), bit for bit."""
    u, f, g = mh.debug_rng(case["seed"], case["subsequence"], 16, rng=1)
    assert [int(x) for x in u] == case["u32"]
    assert [int(x) for x in f.view(np.uint32)] == case["uniform_bits"]
    assert [int(x) for x in g.view(np.uint32)] == case["normal_bits"]


@pytest.mark.parametrize("case", GOLDEN["chains_xorwow"], ids=lambda c: f"{c['room']}{c['n']}")
def test_golden_chains_xorwow_hip(mh, hiplib, case):
    room = MAKE_GOLDEN.make_room(mh, case)
    pts, costs = mh.kernel_wrapper(room, case["chains"], case["steps"], seed=case["seed"], rng=1)
    assert MAKE_GOLDEN.sha(pts) == case["points_sha256"]
    assert MAKE_GOLDEN.sha(costs) == case["costs_sha256"]


@pytest.mark.parametrize("step", STEPS)
@pytest.mark.parametrize("kind,n,chains,steps", [
    ("main", 32, 128, 300),
    ("frozen", 16, 128, 400),
    ("syn", 9, 256, 500),
    ("syn", 64, 64, 1200),   # two launches: the XORWOW state is saved and resumed
    ("syn", 100, 16, 120),
])
def test_xorwow_chains_match_oracle(mh, orc, hiplib, monkeypatch, step, kind, n, chains, steps):
    """Chains seeded exactly as the reference seeds them (curand_init(seed + c, c, 0),
    Kernel.cu:159,943) against the oracle, bit for bit, for both step kernels."""
    kind_ = _use_step(monkeypatch, step, n)
    room = _room(mh, kind, n)
    seed = 1760000000 + n
    with mh.Session(room, chains, seed=seed, rng=1) as s:
        assert s.step_kernel()[2] == kind_  # (never the few-chains instance)
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
    ref_state, ref_costs, _ = orc.run_chains(room, chains, steps, seed, threads=8, rng=1)
    check_chains(f"xorwow {step} {kind} N={n}", pts, costs, ref_state, ref_costs)


def test_xorwow_sharded_sessions_equal_one(mh, hiplib):
    """Chain c's XORWOW stream depends only on its global id: two sessions over [0, 96) and
    [96, 256) reproduce one session over [0, 256) (the multi-GPU sharding invariant)."""
    room = mh.synthetic_room(16)
    seed, steps = 99, 300
    with mh.Session(room, 256, seed=seed, rng=1, track=2) as s:
        s.run(steps)
        s.finalize()
        p_all, c_all = s.download()
    parts = []
    for off, cnt in ((0, 96), (96, 160)):
        with mh.Session(room, cnt, seed=seed, rng=1, track=2, chain_offset=off) as s:
            s.run(steps)
            s.finalize()
            parts.append(s.download())
    assert np.array_equal(np.concatenate([p[0] for p in parts]).view(np.uint32),
                          p_all.view(np.uint32))
    assert np.array_equal(np.concatenate([p[1] for p in parts]).view(np.uint32),
                          c_all.view(np.uint32))


# ---- size limits ---------------------------------------------------------------------------

@pytest.mark.parametrize("step", ["incremental", "full"])
@pytest.mark.parametrize("n", [511, 512])
def test_maximum_room_size(mh, orc, hiplib, monkeypatch, step, n):
    """The largest rooms the library accepts (64 lanes x 8 objects per lane = 512): both step
    kernels against the oracle, bit for bit."""
    monkeypatch.setenv("MH_DELTA", "1" if step == "incremental" else "0")
    room = mh.synthetic_room(n)
    chains, steps, seed = 8, 30, 512
    with mh.Session(room, chains, seed=seed) as s:
        assert s.step_kernel()[2].split("-")[0] == step
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
    ref_pts, ref_costs, _ = orc.run_chains(room, chains, steps, seed, threads=8)
    assert np.array_equal(pts.view(np.uint32), ref_pts.view(np.uint32))
    assert np.array_equal(costs.view(np.uint32), ref_costs.view(np.uint32))


def test_oversized_room_is_rejected(mh, hiplib):
    room = mh.synthetic_room(513)
    with pytest.raises(mh.MHError, match="too large"):
        mh.kernel_wrapper(room, 4, 10, seed=1)


# ---- parallel tempering (mh_options.n_temps > 1) ---------------------------------------------

@pytest.mark.parametrize("step", STEPS)
@pytest.mark.parametrize("kind,n,K,chains,steps,interval", [
    ("main", 32, 4, 64, 300, 25),
    ("syn", 9, 2, 128, 400, 1),       # an exchange round after every step
    ("syn", 16, 8, 64, 1200, 250),    # rounds and 1000-step launches interleave
    ("frozen", 16, 3, 48, 300, 7),
    ("syn", 64, 4, 32, 400, 100),
])
def test_tempering_matches_oracle(mh, orc, hiplib, monkeypatch, step, kind, n, K, chains, steps,
                                  interval):
    """Replica exchange on the device (per-chain beta in both step kernels, mh_exchange_kernel
    between launches) against the oracle's restatement, bit for bit, outputs in rung order."""
    kind_ = _use_step(monkeypatch, step, n)
    room = _room(mh, kind, n)
    seed = 3100 + n + K
    with mh.Session(room, chains, seed=seed, temps=K, swap_interval=interval, beta_min=0.2) as s:
        assert s.step_kernel()[2] == kind_  # (never the few-chains instance)
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
    ref_state, ref_costs, _ = orc.run_chains(room, chains, steps, seed, threads=8, temps=K,
                                             swap_interval=interval, beta_min=0.2)
    check_chains(f"tempering {step} {kind} N={n} K={K}", pts, costs, ref_state, ref_costs)


def test_tempering_resume_and_wrapper(mh, orc, hiplib):
    """Two session runs (600 + 600 steps) equal one of 1200 (the exchange schedule counts steps
    across calls), KernelWrapperEx with the same options equals the session, and tempering with
    best-of-chain tracking and the XORWOW stream together matches the oracle."""
    room = mh.synthetic_room(24)
    K, chains, seed, iv = 4, 64, 51, 150
    with mh.Session(room, chains, seed=seed, temps=K, swap_interval=iv, beta_min=0.5) as s:
        s.run(1200)
        s.finalize()
        p1, c1 = s.download()
    with mh.Session(room, chains, seed=seed, temps=K, swap_interval=iv, beta_min=0.5) as s:
        s.run(600)
        s.run(600)
        s.finalize()
        p2, c2 = s.download()
    assert np.array_equal(p1.view(np.uint32), p2.view(np.uint32))
    assert np.array_equal(c1.view(np.uint32), c2.view(np.uint32))
    p3, c3 = mh.kernel_wrapper(room, chains, 1200, seed=seed, temps=K, swap_interval=iv,
                               beta_min=0.5)
    assert np.array_equal(p1.view(np.uint32), p3.view(np.uint32))
    p4, c4 = mh.kernel_wrapper(room, chains, 500, seed=seed, temps=K, swap_interval=iv,
                               beta_min=0.5, track=2, rng=1)
    st, rc, _ = orc.run_chains(room, chains, 500, seed, threads=8, temps=K, swap_interval=iv,
                               beta_min=0.5, track=2, rng=1)
    assert np.array_equal(p4.view(np.uint32), st.astype(np.float32).view(np.uint32))
    assert np.array_equal(c4.view(np.uint32), rc.view(np.uint32))


def test_tempering_validation(mh, hiplib):
    room = mh.synthetic_room(8)
    with pytest.raises(mh.MHError, match="multiple of n_temps"):
        mh.kernel_wrapper(room, 10, 10, seed=1, temps=4, swap_interval=5, beta_min=0.5)
    with pytest.raises(mh.MHError, match="beta_min"):
        mh.kernel_wrapper(room, 8, 10, seed=1, temps=4, swap_interval=5, beta_min=3.0)


@pytest.mark.parametrize("step", ["full", "incremental"])
def test_wave_rng_window_overrun(mh, orc, hiplib, monkeypatch, step):
    """A 64-object room with 61 objects frozen: a pick redraws ~20 times on average, so steps
    regularly draw past WaveRng's 64-word window (the direct-draw fallback for words and
    normals). Bit for bit against the oracle, including across launch boundaries."""
    monkeypatch.setenv("MH_DELTA", "1" if step == "incremental" else "0")
    room = mh.synthetic_room(64)
    for i in range(61):
        room.cfg[i].frozen = True
    chains, steps, seed = 64, 1300, 606
    with mh.Session(room, chains, seed=seed) as s:
        assert s.step_kernel()[:1] == (64,) and s.step_kernel()[2].split("-")[0] == step
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
    ref_pts, ref_costs, _ = orc.run_chains(room, chains, steps, seed, threads=8)
    assert np.array_equal(pts.view(np.uint32), ref_pts.view(np.uint32))
    assert np.array_equal(costs.view(np.uint32), ref_costs.view(np.uint32))


@pytest.mark.parametrize("step", ["full", "incremental"])
@pytest.mark.parametrize("n,chains,steps", [(20, 256, 600), (64, 128, 500), (200, 16, 80)])
def test_stacked_objects_symmetry_ties(mh, orc, hiplib, monkeypatch, step, n, chains, steps):
    """Half the objects stacked on one pose, every other one of them frozen: the symmetry rows
    keep exactly tied estimates in their columns for the whole run, so the row-leader test
    (group_sym_lead) must see the tie and fall back to the exact scan at every step."""
    monkeypatch.setenv("MH_DELTA", "1" if step == "incremental" else "0")
    room = mh.synthetic_room(n)
    p0 = room.cfg[0]
    for i in range(1, n // 2):
        room.cfg[i].x, room.cfg[i].y, room.cfg[i].rotY = p0.x, p0.y, p0.rotY
        room.cfg[i].frozen = i % 2 == 1
    seed = 8800 + n
    with mh.Session(room, chains, seed=seed) as s:
        assert s.step_kernel()[2].split("-")[0] == step
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
    ref_pts, ref_costs, _ = orc.run_chains(room, chains, steps, seed, threads=8)
    check_chains(f"{step} stacked N={n}", pts, costs, ref_pts, ref_costs)


@pytest.mark.parametrize("step", ["full", "incremental"])
@pytest.mark.parametrize("slack", ["1", "4", "64", "1e6"])
@pytest.mark.parametrize("kind,n,chains,steps", [
    ("syn", 64, 64, 1200),   # config 3's room; two launches (the lazy costs cross a launch end)
    ("main", 32, 64, 600),
    ("wrap", 24, 64, 500),
    ("syn", 9, 64, 500),
    ("syn", 256, 16, 1200),  # config 5's room: the incremental kernel's 4-slot instance
])
def test_bound_decision_paths(mh, orc, hiplib, monkeypatch, step, slack, kind, n, chains, steps):
    """The step bound decides Accept without the exact costs where it can: a certain reject or
    a certain accept that leaves the current total known only as an interval (both step kernels;
    the full-evaluation kernel with one object per lane); otherwise the exact costs are computed,
    the current configuration's too when they are pending. $MH_BOUND_SLACK widens the bound's error
    allowance (still a valid bound), which moves steps from the certain decisions to the exact
    paths: every mix must give the oracle's chains."""
    monkeypatch.setenv("MH_BOUND_SLACK", slack)
    kind_ = _use_step(monkeypatch, step, n)
    room = _room(mh, kind, n)
    seed = 9100 + n
    with mh.Session(room, chains, seed=seed) as s:
        assert s.step_kernel()[2].split("-")[0] == kind_
        s.run(steps)
        cur = s.current_costs()
        s.finalize()
        pts, costs = s.download()
    ref_pts, ref_costs, _ = orc.run_chains(room, chains, steps, seed, threads=8)
    check_chains(f"slack {slack} {step} {kind} N={n}", pts, costs, ref_pts, ref_costs)
    # the costs carried between launches are the exact ones (all but OffLimits, which the step
    # path does not evaluate)
    keep = [1, 2, 3, 4, 5, 7]
    assert np.array_equal(cur[:, keep].view(np.uint32), costs[:, keep].view(np.uint32))
