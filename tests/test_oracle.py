"""The oracle (oracle/mh_oracle.c) pinned against the reference's known answers, plus
hand-derived analytic cases and the defined chain semantics. CPU only.

Pins:
  * the reference's own Costs() on the main() fixture (Kernel.cu:1007-1166),
    all eight components to 9 significant digits.
  * Random123 known-answer vectors for philox4x32 with 10 rounds (the generator behind
    rocRAND's rocrand_state_philox4x32_10).
"""
import ctypes as C
import math

import numpy as np
import pytest

PI = 3.1416
KAT = {"totalCosts": 3921.14038, "PairWiseCosts": 0.0, "VisualBalanceCosts": -65.7609329,
       "FocalPointCosts": 36.7696877, "SymmetryCosts": 46.1316452, "ClearanceCosts": 16.0,
       "OffLimitsCosts": 0.0, "SurfaceAreaCosts": 3888.0}


def test_known_answer_main_fixture(mh, orc):
    got = orc.costs(mh.main_fixture())
    for k, name in enumerate(mh.COST_FIELDS):
        assert got[k] == pytest.approx(KAT[name], rel=1e-8, abs=1e-12), name


@pytest.mark.parametrize("ctr,key,out", [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox_random123_kat(orc, ctr, key, out):
    lib = orc.load()
    o = (C.c_uint32 * 4)()
    lib.orc_philox4x32_10((C.c_uint32 * 4)(*ctr), (C.c_uint32 * 2)(*key), o)
    assert tuple(o) == out


def test_stream_is_rocrand_layout(orc):
    """rocRAND philox4x32_10: key = seed, counter = (block, 0, subsequence lo, hi)."""
    lib = orc.load()
    seed, sub = 0x0123456789ABCDEF, 0x00000002_00000007
    u, _, _ = orc.rng_streams(seed, sub, 12)
    key = (C.c_uint32 * 2)(seed & 0xffffffff, seed >> 32)
    for blk in range(3):
        o = (C.c_uint32 * 4)()
        lib.orc_philox4x32_10((C.c_uint32 * 4)(blk, 0, sub & 0xffffffff, sub >> 32), key, o)
        assert tuple(u[4 * blk:4 * blk + 4]) == tuple(o)


def _rng_with_words(orc, words):
    """An orc_rng whose next draws are `words` (first four), as a device stream would give."""
    r = orc.OrcRng()
    for k in range(4):
        r.result[k] = words[k]
    r.substate = 0
    return r


def test_uniform_conversion(orc):
    lib = orc.load()
    r = _rng_with_words(orc, [0, 0xFFFFFFFF, 0xFFFFFF80, 0x80000000])
    vals = [lib.orc_rng_uniform(C.byref(r)) for _ in range(4)]
    assert vals[0] == np.float32(2.3283064e-10)
    assert vals[1] == 1.0 and vals[2] == 1.0       # u == 1.0f happens (Kernel.cu:569)
    assert vals[3] == pytest.approx(0.5, abs=1e-9)


def test_index_n_is_redrawn(mh, orc):
    """generateRandomIntInRange(N-1, 0) with u == 1.0f returns N for N >= 33 (Kernel.cu:571);
    the defined chain treats index N as frozen and redraws."""
    lib = orc.load()
    r = _rng_with_words(orc, [0xFFFFFFFF] * 4)
    assert lib.orc_rand_int(C.byref(r), 63, 0) == 64
    r = _rng_with_words(orc, [0xFFFFFFFF] * 4)
    assert lib.orc_rand_int(C.byref(r), 31, 0) == 31       # N = 32: no overflow
    room = mh.synthetic_room(64)
    r = _rng_with_words(orc, [0xFFFFFFFF, 0xFFFFFFFF, 0x40000000, 0])
    k = lib.orc_pick_object(C.cast(room.cfg, C.c_void_p), 64, C.byref(r))
    assert k == int(np.float32(np.float32(0.25) * np.float32(63.999999)))  # third draw used
    frozen = mh.synthetic_room(16, freeze_every=2)   # odd objects frozen
    r = _rng_with_words(orc, [0x18000000, 0x28000000, 0, 0])  # picks 1 (frozen), then 2
    k = lib.orc_pick_object(C.cast(frozen.cfg, C.c_void_p), 16, C.byref(r))
    assert frozen.cfg[1].frozen and k == 2


def test_index_n_needs_33_objects(orc):
    """The index-n pick exists only from 33 objects up: u == 1.0f (the largest uniform; the
    result grows with u) gives generateRandomIntInRange(N-1, 0) = N - 1 for every N <= 32 and N
    for N = 33..256, where N - 1 + 0.999999 rounds up to the float N (Kernel.cu:566-574). So the
    speculative kernel (N <= 8) never meets it."""
    lib = orc.load()
    for n in range(1, 257):
        r = _rng_with_words(orc, [0xFFFFFFFF] * 4)
        assert lib.orc_rand_int(C.byref(r), n - 1, 0) == (n if n >= 33 else n - 1), n


def test_swap_with_itself_rounds_to_float(mh, orc):
    """Swap (Kernel.cu:655-703) with obj1 == obj2: obj1's pose goes through float temporaries."""
    lib = orc.load()
    room = mh.synthetic_room(4)
    cfg = mh.clone_cfg(room)
    cfg[2].x = 1.0 + 2 ** -40
    cfg[2].rotY = 0.1
    before = [(cfg[i].x, cfg[i].y, cfg[i].rotY) for i in range(4)]
    # mode draw u ~ 0.9 -> p = 2 (swap); both picks u ~ 0.6 -> index 2 of 4
    r = _rng_with_words(orc, [0xE6666666, 0x9999999A, 0x9999999A, 0])
    lib.orc_propose(C.byref(orc.orc_room(room)), C.cast(cfg, C.c_void_p), C.byref(r))
    assert cfg[2].x == float(np.float32(1.0 + 2 ** -40)) == 1.0
    assert cfg[2].rotY == float(np.float32(0.1))
    for i in (0, 1, 3):
        assert (cfg[i].x, cfg[i].y, cfg[i].rotY) == before[i]


def _two_object_room(mh, xy0, xy1, rel=(2.0, 4.0), ang=(PI / 4, 5 * PI / 8)):
    room = mh.main_fixture()
    room.srf.nObjs = 2
    room.srf.nClearances = 0
    room.cfg[0].x, room.cfg[0].y = xy0
    room.cfg[1].x, room.cfg[1].y = xy1
    room.rss[0].TargetRange.targetRangeStart, room.rss[0].TargetRange.targetRangeEnd = rel
    room.rsa[0].angleMin, room.rsa[0].angleMax = ang
    return room


@pytest.mark.parametrize("d,expect", [(1.0, -(1.0 / 2.0) ** 2), (3.0, 0.0), (8.0, -(4.0 / 8.0) ** 2)])
def test_pairwise_term(mh, orc, d, expect):
    """PairWiseCosts, Kernel.cu:210-233: -(d/start)^2 below the range, -(end/d)^2 above."""
    lib = orc.load()
    room = _two_object_room(mh, (0.0, 0.0), (d, 0.0))
    got = lib.orc_pairwise(C.byref(orc.orc_room(room)), C.cast(room.cfg, C.c_void_p))
    assert got == pytest.approx(expect, rel=1e-15, abs=0)


def test_pairwise_angle_term(mh, orc):
    """PairWiseAngleCosts, Kernel.cu:236-263: source at (2,2), target at origin facing 0:
    theta = atan2(2, 2) = pi/4 lies inside [PI/4 - e, 5PI/8]; the reference's condition
    `min < d || d < max` still charges min(|d - min|, |d - max|) / norm."""
    lib = orc.load()
    room = _two_object_room(mh, (2.0, 2.0), (0.0, 0.0), ang=(0.5, 5 * PI / 8))
    got = lib.orc_pairwise_angle(C.byref(orc.orc_room(room)), C.cast(room.cfg, C.c_void_p))
    d = math.atan2(2.0, 2.0)
    norm = (2 * PI - (5 * PI / 8 - 0.5)) / 2.0
    assert got == pytest.approx(-min(abs(d - 0.5), abs(d - 5 * PI / 8)) / norm, rel=1e-12)


def test_visual_balance_term(mh, orc):
    """VisualBalanceCosts, Kernel.cu:191-207: minus the distance from the area-weighted
    centroid to (centroidX/2, centroidY/2)."""
    lib = orc.load()
    room = _two_object_room(mh, (1.0, 1.0), (3.0, 1.0))
    room.cfg[1].length, room.cfg[1].width = 3.0, 1.0  # area 3 vs 1
    room.srf.centroidX, room.srf.centroidY = 4.0, 6.0
    got = lib.orc_visual_balance(C.byref(orc.orc_room(room)), C.cast(room.cfg, C.c_void_p))
    cx, cy = (1 * 1.0 + 3 * 3.0) / 4, (1 * 1.0 + 3 * 1.0) / 4
    assert got == pytest.approx(-math.hypot(cx - 2.0, cy - 3.0), rel=1e-7)


def test_focal_point_term(mh, orc):
    """FocalPointCosts, Kernel.cu:266-281: -sum cos(atan2(fy - y, fx - x) - rotY + PI/2)."""
    lib = orc.load()
    room = _two_object_room(mh, (5.0, 1.0), (1.0, 5.0))
    room.cfg[0].rotY, room.cfg[1].rotY = 0.3, 2.0
    got = lib.orc_focal_point(C.byref(orc.orc_room(room)), C.cast(room.cfg, C.c_void_p))
    exp = -sum(math.cos(math.atan2(5.0 - y, 5.0 - x) - r + PI / 2)
               for x, y, r in [(5.0, 1.0, 0.3), (1.0, 5.0, 2.0)])
    assert got == pytest.approx(exp, rel=1e-6)


def test_clearance_min_value_quirk(mh, orc):
    """minValue keeps vertex 0's x UNtranslated (Kernel.cu:371): an off-limits rectangle
    (2,2),(2,0),(0,0),(0,2) at (5,5) spans x in [2, 7], not [5, 7]. A clearance box
    [3,4]x[5,6] therefore overlaps it by 1 (and would not without the quirk)."""
    lib = orc.load()
    room = mh.main_fixture()
    room.srf.nObjs, room.srf.nClearances = 2, 1
    room.cfg[0].x = room.cfg[0].y = 5.0
    room.cfg[1].x, room.cfg[1].y = 3.0, 5.0
    # clearance 0: unit square (vertices 8..11 are the 2x2 square; use a unit one at 0..3)
    verts = (mh.abi.vertex * 16)()
    C.memmove(verts, room.vertices, C.sizeof(verts))
    for k, (x, y) in enumerate([(1, 1), (1, 0), (0, 0), (0, 1)]):
        verts[k] = mh.abi.vertex(x, y, 0)
    room.vertices = verts
    room.clearances[0] = mh.abi.rectangle(0, 1, 2, 3, 1)   # source object 1 at (3, 5)
    room.offlimits[0] = mh.abi.rectangle(8, 9, 10, 11, 0)  # 2x2 square at (5, 5)
    room.offlimits[1] = mh.abi.rectangle(4, 5, 6, 7, 0)    # (3,2),(3,0),(1,0),(1,2) at (3,5)
    got = lib.orc_clearance(C.byref(orc.orc_room(room)), C.cast(room.cfg, C.c_void_p))
    # The clearance box is itself quirked: v0.x = 1 untranslated -> [1, 4] x [5, 6].
    # j=0: [2,7]x[5,7] -> [2,4]x[5,6] = 2;  j=1: v0.x = 3 untranslated -> [3,6]x[5,7] -> 1.
    # Without the quirk the boxes would be [3,4], [5,7], [4,6] in x: no overlap at all.
    assert got == -3.0


def test_surface_area_uses_cfg_i_for_clearances(mh, orc):
    """SurfaceAreaCosts translates clearance i by cfg[i], not cfg[SourceIndex] (Kernel.cu:456)."""
    lib = orc.load()
    room = mh.main_fixture()
    room.srf.nObjs, room.srf.nClearances = 2, 1
    room.cfg[0].x = room.cfg[0].y = 5.0        # cfg[0]: inside
    room.cfg[1].x, room.cfg[1].y = 9.5, 5.0    # source object: near the right wall
    room.clearances[0] = mh.abi.rectangle(0, 1, 2, 3, 1)
    got = lib.orc_surface_area(C.byref(orc.orc_room(room)), C.cast(room.cfg, C.c_void_p))
    # clearance 0 is the 2x2 square (vertices 0..3) placed at cfg[0] = (5,5): inside -> 0.
    # object 1's off-limits (3,2),(3,0),(1,0),(1,2) at (9.5,5): x in [3, 12.5] -> 2.5 x 2 outside
    assert got == -5.0


def test_total_excludes_off_limits(mh, orc):
    room = mh.synthetic_room(16)
    c = orc.costs(room)
    assert c[6] != 0.0
    t = np.float32(c[1]) + np.float32(c[2])
    for k in (3, 4, 5, 7):
        t = np.float32(t + np.float32(c[k]))
    assert c[0] == t


def test_pairwise_is_product_of_distance_and_angle(mh, orc):
    lib = orc.load()
    room = mh.synthetic_room(12)
    rm, cfg = C.byref(orc.orc_room(room)), C.cast(room.cfg, C.c_void_p)
    prod = np.float32(lib.orc_pairwise(rm, cfg) * lib.orc_pairwise_angle(rm, cfg))
    assert orc.costs(room)[1] == np.float32(room.srf.WeightPairWise) * prod


def test_chain_determinism_and_shards(mh, orc):
    room = mh.synthetic_room(10)
    a = orc.run_chains(room, 12, 60, seed=3, threads=3)
    b = orc.run_chains(room, 12, 60, seed=3, threads=1)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    # chain c draws subsequence c: a shard [4, 12) equals the tail of the full run
    s = orc.run_chains(room, 8, 60, seed=3, chain_begin=4)
    assert np.array_equal(s[0], a[0][4:]) and np.array_equal(s[1], a[1][4:])
    assert len({a[0][i].tobytes() for i in range(12)}) == 12


def test_zero_iterations_returns_input(mh, orc):
    room = mh.main_fixture()
    pts, costs, acc = orc.run_chains(room, 3, 0, seed=1)
    base = np.ctypeslib.as_array(room.cfg)
    assert np.array_equal(pts[1, :, 0], base["x"].astype(np.float32))
    assert np.array_equal(costs[0], orc.costs(room)) and not acc.any()


def test_validation_errors(mh, orc):
    lib = orc.load()
    room = mh.synthetic_room(8, freeze_every=1)  # every object frozen
    assert lib.orc_validate(C.byref(orc.orc_room(room)), C.cast(room.cfg, C.c_void_p)) != 0
    assert b"frozen" in lib.orc_last_error()
    room = mh.synthetic_room(8)
    room.rss[0].TargetIndex = 8
    assert lib.orc_validate(C.byref(orc.orc_room(room)), C.cast(room.cfg, C.c_void_p)) != 0
    room = mh.synthetic_room(8)
    room.srf.nClearances = 9
    assert lib.orc_validate(C.byref(orc.orc_room(room)), C.cast(room.cfg, C.c_void_p)) != 0


def test_accept_rule(orc):
    """Accept (Kernel.cu:706-713): u < min(1, exp(2 (star - cur))) -- maximisation."""
    lib = orc.load()
    r = _rng_with_words(orc, [0x80000000] * 4)                    # u = 0.5
    assert lib.orc_accept(10.0, 10.0, C.byref(r)) == 1            # exp(0) = 1 > 0.5
    r = _rng_with_words(orc, [0x80000000] * 4)
    assert lib.orc_accept(10.0 - 0.5 * math.log(2) - 1e-3, 10.0, C.byref(r)) == 0
    r = _rng_with_words(orc, [0xFFFFFFFF] * 4)                    # u = 1.0f: never accepts
    assert lib.orc_accept(1e6, 0.0, C.byref(r)) == 0


def _copy(arr):
    out = (arr._type_ * len(arr))()
    C.memmove(out, arr, C.sizeof(out))
    return out


@pytest.mark.parametrize("track", [1, 2])
def test_best_of_chain_restatement(mh, orc, track):
    """orc_run_chains_ex's best-of-chain tracking against the reference's commented-out loop
    (Kernel.cu:779-782, 808-816), re-walked step by step here through orc_propose / orc_costs /
    orc_accept: best starts as the initial configuration, every star is compared before Accept
    with a strict comparison, and the output is cfgBest with bestCosts."""
    lib = orc.load()
    room = mh.synthetic_room(8)
    n, steps, seed, chains = room.n, 120, 31337, 3
    ref_state, ref_costs, _ = orc.run_chains(room, chains, steps, seed, track=track)
    better = (lambda s, b: s < b) if track == 1 else (lambda s, b: s > b)
    orm = orc.orc_room(room)
    for c in range(chains):
        rng = orc.OrcRng()
        lib.orc_rng_init(C.byref(rng), seed, c)
        cur = mh.clone_cfg(room)
        cc = orc.costs(room, cur)
        best, bc = _copy(cur), cc.copy()
        for _ in range(steps):
            star = _copy(cur)
            lib.orc_propose(C.byref(orm), C.cast(star, C.c_void_p), C.byref(rng))
            sc = orc.costs(room, star)
            if better(sc[0], bc[0]):
                best, bc = _copy(star), sc
            if lib.orc_accept(float(sc[0]), float(cc[0]), C.byref(rng)):
                cur, cc = star, sc
        got = np.array([[b.x, b.y, b.z, b.rotX, b.rotY, b.rotZ] for b in best])
        assert np.array_equal(got, ref_state[c])
        assert np.array_equal(bc.view(np.uint32), ref_costs[c].view(np.uint32))


def test_best_of_chain_bounds(mh, orc):
    """Lowest <= initial and final; highest >= initial and final; the reported costs are the
    costs of the reported configuration."""
    room = mh.synthetic_room(16)
    chains, steps, seed = 16, 400, 5
    init = orc.costs(room)[0]
    _, fin, _ = orc.run_chains(room, chains, steps, seed, threads=4)
    lo_s, lo, _ = orc.run_chains(room, chains, steps, seed, threads=4, track=1)
    hi_s, hi, _ = orc.run_chains(room, chains, steps, seed, threads=4, track=2)
    assert np.all(lo[:, 0] <= init) and np.all(lo[:, 0] <= fin[:, 0])
    assert np.all(hi[:, 0] >= init) and np.all(hi[:, 0] >= fin[:, 0])
    base = np.ctypeslib.as_array(room.cfg)
    for c in (0, chains - 1):
        cfg = mh.clone_cfg(room)
        for i in range(room.n):
            cfg[i].x, cfg[i].y, cfg[i].z, cfg[i].rotX, cfg[i].rotY, cfg[i].rotZ = hi_s[c, i]
            assert cfg[i].frozen == base[i]["frozen"]
        assert np.array_equal(orc.costs(room, cfg).view(np.uint32), hi[c].view(np.uint32))


def test_xorwow_curand_formulas(orc):
    """cuRAND XORWOW restated by hand: _curand_init_scratch's seeding of seed 0, one step of the
    recurrence plus the Weyl sequence, and curand_uniform = x * 2^-32 + 2^-33 in float.
    (The subsequence jump is pinned against rocRAND's engine in test_golden.py.)"""
    lib = orc.load()
    r = orc.rng_init(123, 0, orc.XORWOW_CURAND)
    d, x = r.xw[0], list(r.xw)[1:]
    v = lib.orc_rng_next(C.byref(r))
    t = (x[0] ^ (x[0] >> 2)) & 0xffffffff
    x4 = (x[4] ^ (x[4] << 4) ^ t ^ (t << 1)) & 0xffffffff
    assert v == (d + 362437 + x4) & 0xffffffff
    r = orc.rng_init(123, 0, orc.XORWOW_CURAND)
    w = lib.orc_rng_next(C.byref(r))
    r = orc.rng_init(123, 0, orc.XORWOW_CURAND)
    assert lib.orc_rng_uniform(C.byref(r)) == np.float32(np.float32(w) * np.float32(2**-32) +
                                                          np.float32(2**-33))
    a = orc.rng_init(5, 3, orc.XORWOW_CURAND)
    b = orc.rng_init(5, 1, orc.XORWOW_CURAND)
    c = orc.rng_init(5, 2, orc.XORWOW_CURAND)
    assert list(a.xw) != list(b.xw) != list(c.xw)
    # cuRAND seeding of seed 0 by hand (_curand_init_scratch)
    z = orc.rng_init(0, 0, orc.XORWOW_CURAND)
    t0 = (1099087573 * 0xaad26b49) & 0xffffffff
    t1 = (2591861531 * 0xf7dcefdd) & 0xffffffff
    assert list(z.xw) == [(6615241 + t1 + t0) & 0xffffffff, (123456789 + t0) & 0xffffffff,
                          362436069 ^ t0, (521288629 + t1) & 0xffffffff, 88675123 ^ t1,
                          (5783321 + t0) & 0xffffffff]


def _ladder(K, beta_min):
    return [2.0 if k == 0 else 2.0 * math.pow(beta_min / 2.0, k / (K - 1)) for k in range(K)]


@pytest.mark.parametrize("K,interval,steps", [(3, 5, 31), (4, 1, 12), (2, 40, 40)])
def test_tempering_restatement(mh, orc, K, interval, steps):
    """orc_run_chains_ex's parallel tempering against the rule written out here step by step
    (include/mh_kernel.h KernelWrapperEx): replicas step at their rung's beta; after every
    `interval` steps round t tries the pairs (k, k+1), k = (t-1) mod 2 + 2i, with the Philox
    uniform of (seed, 2^63 + group, (t-1)*K + k); outputs land in rung order."""
    lib = orc.load()
    room = mh.synthetic_room(8)
    seed, groups, beta_min = 77, 2, 0.25
    chains = groups * K
    st, costs, acc = orc.run_chains(room, chains, steps, seed, temps=K, swap_interval=interval,
                                    beta_min=beta_min)
    lad = _ladder(K, beta_min)
    orm = orc.orc_room(room)
    for g in range(groups):
        reps = []
        for j in range(K):
            r = orc.rng_init(seed, g * K + j)
            cur = mh.clone_cfg(room)
            reps.append({"r": r, "cur": cur, "cc": orc.costs(room, cur), "rung": j})
        perm = list(range(K))
        done = 0
        while done < steps:
            chunk = min(steps - done, interval - done % interval)
            for rep_ in reps:
                for _ in range(chunk):
                    star = _copy(rep_["cur"])
                    lib.orc_propose(C.byref(orm), C.cast(star, C.c_void_p), C.byref(rep_["r"]))
                    sc = orc.costs(room, star)
                    if lib.orc_accept_at(float(sc[0]), float(rep_["cc"][0]), lad[rep_["rung"]],
                                         C.byref(rep_["r"])):
                        rep_["cur"], rep_["cc"] = star, sc
            done += chunk
            if done % interval == 0:
                t = done // interval
                for k in range((t - 1) % 2, K - 1, 2):
                    a, b = perm[k], perm[k + 1]
                    ur = orc.OrcRng()
                    lib.orc_rng_init_offset(C.byref(ur), seed, (1 << 63) | g, (t - 1) * K + k)
                    u = lib.orc_rng_uniform(C.byref(ur))
                    thr = min(np.float32(1.0), np.float32(math.exp(
                        (lad[k] - lad[k + 1]) * (float(reps[b]["cc"][0]) - float(reps[a]["cc"][0])))))
                    if np.float32(u) < thr:
                        perm[k], perm[k + 1] = b, a
                        reps[a]["rung"], reps[b]["rung"] = k + 1, k
        for j, rep_ in enumerate(reps):
            slot = g * K + rep_["rung"]
            got = np.array([[b.x, b.y, b.z, b.rotX, b.rotY, b.rotZ] for b in rep_["cur"]])
            assert np.array_equal(got, st[slot])
            assert np.array_equal(rep_["cc"].view(np.uint32), costs[slot].view(np.uint32))


def test_tempering_at_one_temperature_permutes_plain_chains(mh, orc):
    """With beta_min = BETA every rung runs the reference's chain, so every exchange is accepted
    (threshold 1) and the outputs are the plain chains, permuted within each group."""
    room = mh.synthetic_room(16)
    K, chains, steps, seed = 4, 16, 60, 9
    st, costs, _ = orc.run_chains(room, chains, steps, seed, temps=K, swap_interval=7,
                                  beta_min=2.0)
    pst, pcosts, _ = orc.run_chains(room, chains, steps, seed, state=True)
    for g in range(chains // K):
        a = sorted(costs[g * K:(g + 1) * K].view(np.uint32).tolist())
        b = sorted(pcosts[g * K:(g + 1) * K].view(np.uint32).tolist())
        assert a == b


@pytest.mark.parametrize("kw", [{}, {"track": 2}, {"temps": 4, "swap_interval": 7},
                                {"rng": 1}], ids=["plain", "track", "tempering", "xorwow"])
def test_step_offlimits_knob_keeps_outputs(mh, orc, kw):
    """set_step_offlimits(False) leaves OffLimits out of the per-step Costs() (it never enters
    totalCosts, Kernel.cu:547) and evaluates it for the output configurations only: every
    output -- poses, all eight costs, accept counts -- is the same bit for bit."""
    room = mh.synthetic_room(24)
    a = orc.run_chains(room, 8, 150, 31, threads=4, **kw)
    orc.set_step_offlimits(False)
    try:
        b = orc.run_chains(room, 8, 150, 31, threads=4, **kw)
    finally:
        orc.set_step_offlimits(True)
    for x, y in zip(a, b):
        x, y = np.asarray(x), np.asarray(y)
        assert x.dtype == y.dtype and np.array_equal(x.view(np.uint8), y.view(np.uint8))
    assert np.any(a[1][:, 6] != 0)  # the room's objects do overlap: OffLimits is exercised


def test_u1_accept_fixture_exercises_the_edge(mh, orc):
    """The u == 1.0f fixtures (tests/golden/find_u1_accept.py) do draw Accept's u == 1.0f
    against an uphill proposal in the oracle, at the recorded step and not before."""
    import json
    from pathlib import Path
    g = json.loads((Path(__file__).with_name("golden") / "golden.json").read_text())
    assert g["u1_accept"]
    for case in g["u1_accept"]:
        room = mh.synthetic_room(case["n"])
        for steps, expect in ((case["step"] - 1, 0), (case["step"], 1)):
            orc.u1_uphill_draws(reset=True)
            orc.run_chains(room, 1, steps, case["seed"], chain_begin=case["chain"])
            assert orc.u1_uphill_draws() == expect, (case, steps)
