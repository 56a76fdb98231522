"""TEST INFRASTRUCTURE ONLY: ctypes loader for the C restatement in mh_oracle.c.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module. The
product (libmhgpu.so) never loads it.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "_build" / "liboracle.so"
SOURCES = [ORACLE_DIR / "mh_oracle.c"]
# the shared transcendentals (the only product file the oracle includes besides the wire structs)
MATH_HEADER = ORACLE_DIR.parent / "metropolis-hastings-gpgpu_amd" / "csrc" / "mh_math.h"
CFLAGS = ["-O2", "-std=c11", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
          "-pthread"]

_lib = None


def build(force: bool = False) -> Path:
    import subprocess
    LIB_PATH.parent.mkdir(parents=True, exist_ok=True)
    newest = max(p.stat().st_mtime for p in SOURCES + [ORACLE_DIR / "mh_oracle.h", MATH_HEADER,
                                                        ORACLE_DIR.parent / "include" / "mh_kernel.h"])
    if force or not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < newest:
        cmd = ["gcc", *CFLAGS, *map(str, SOURCES), "-o", str(LIB_PATH), "-lm"]
        subprocess.run(cmd, check=True)
    return LIB_PATH


def load(pkg=None) -> C.CDLL:
    """Loads liboracle.so (building it with gcc if needed). `pkg` is the product package whose
    ctypes struct mirrors are reused for the argument types."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        build()
    lib = C.CDLL(str(LIB_PATH))
    P = C.POINTER
    lib.orc_costs.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.orc_costs.restype = None
    lib.orc_validate.argtypes = [C.c_void_p, C.c_void_p]
    lib.orc_validate.restype = C.c_int
    lib.orc_last_error.restype = C.c_char_p
    for name, rt in [("orc_visual_balance", C.c_double), ("orc_pairwise", C.c_double),
                     ("orc_pairwise_angle", C.c_double), ("orc_focal_point", C.c_double),
                     ("orc_symmetry", C.c_float), ("orc_clearance", C.c_float),
                     ("orc_surface_area", C.c_float), ("orc_off_limits", C.c_float)]:
        f = getattr(lib, name)
        f.argtypes = [C.c_void_p, C.c_void_p]
        f.restype = rt
    lib.orc_philox_stream.argtypes = [C.c_uint64, C.c_uint64, P(C.c_uint32), C.c_int]
    lib.orc_philox_stream.restype = None
    lib.orc_philox4x32_10.argtypes = [P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)]
    lib.orc_philox4x32_10.restype = None
    lib.orc_rng_init.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64]
    lib.orc_rng_init_xorwow.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_int]
    lib.orc_rng_init_xorwow.restype = None
    lib.orc_rng_init_offset.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64]
    lib.orc_rng_init_offset.restype = None
    lib.orc_rng_next.argtypes = [C.c_void_p]
    lib.orc_rng_next.restype = C.c_uint32
    lib.orc_rng_uniform.argtypes = [C.c_void_p]
    lib.orc_rng_uniform.restype = C.c_float
    lib.orc_rng_normal.argtypes = [C.c_void_p]
    lib.orc_rng_normal.restype = C.c_float
    lib.orc_run_chains.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int64, C.c_int64,
                                   C.c_int, C.c_int, C.c_void_p, C.c_void_p, P(C.c_int64)]
    lib.orc_run_chains.restype = C.c_int
    lib.orc_run_chains_state.argtypes = lib.orc_run_chains.argtypes
    lib.orc_run_chains_state.restype = C.c_int
    lib.orc_run_chains_ex.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64,
                                      C.c_int, C.c_int, C.c_void_p, C.c_void_p, P(C.c_int64)]
    lib.orc_run_chains_ex.restype = C.c_int
    lib.orc_rand_int.argtypes = [C.c_void_p, C.c_int, C.c_int]
    lib.orc_rand_int.restype = C.c_int
    lib.orc_pick_object.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    lib.orc_pick_object.restype = C.c_int
    lib.orc_index_n_draws.argtypes = [C.c_int]
    lib.orc_index_n_draws.restype = C.c_longlong
    lib.orc_u1_uphill_draws.argtypes = [C.c_int]
    lib.orc_u1_uphill_draws.restype = C.c_longlong
    lib.orc_set_step_offlimits.argtypes = [C.c_int]
    lib.orc_set_step_offlimits.restype = None
    lib.orc_propose.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.orc_accept.argtypes = [C.c_double, C.c_double, C.c_void_p]
    lib.orc_accept.restype = C.c_int
    lib.orc_accept_at.argtypes = [C.c_double, C.c_double, C.c_double, C.c_void_p]
    lib.orc_accept_at.restype = C.c_int
    lib.orc_math_apply.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    lib.orc_math_apply.restype = C.c_int
    for name in ("orc_math_eval", "orc_math_eval_libm"):
        f = getattr(lib, name)
        f.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_int, C.c_void_p]
        f.restype = C.c_int
    _lib = lib
    return lib


class OrcRoom(C.Structure):
    _fields_ = [("rs", C.c_void_p), ("ra", C.c_void_p), ("clearances", C.c_void_p),
                ("offlimits", C.c_void_p), ("vertices", C.c_void_p),
                ("surfaceRectangle", C.c_void_p), ("srf", C.c_void_p)]


class OrcRng(C.Structure):
    _fields_ = [("counter", C.c_uint32 * 4), ("result", C.c_uint32 * 4), ("key", C.c_uint32 * 2),
                ("substate", C.c_uint32), ("bm_has", C.c_int32), ("bm_val", C.c_float),
                ("kind", C.c_int32), ("xw", C.c_uint32 * 6)]


PHILOX, XORWOW_CURAND, XORWOW_ROCRAND = 0, 1, 2


def orc_room(room) -> OrcRoom:
    """Wraps a product Room (ctypes arrays) for the oracle; keeps `room` alive via ._keep."""
    r = OrcRoom(C.cast(room.rss, C.c_void_p), C.cast(room.rsa, C.c_void_p),
                C.cast(room.clearances, C.c_void_p), C.cast(room.offlimits, C.c_void_p),
                C.cast(room.vertices, C.c_void_p), C.cast(room.surface_rectangle, C.c_void_p),
                C.cast(C.pointer(room.srf), C.c_void_p))
    r._keep = room
    return r


def costs(room, cfg=None) -> np.ndarray:
    """orc_costs -> float32[8] in resultCosts order."""
    lib = load()
    out = (C.c_float * 8)()
    lib.orc_costs(C.byref(orc_room(room)), C.cast(room.cfg if cfg is None else cfg, C.c_void_p),
                  out)
    return np.frombuffer(bytes(out), dtype=np.float32).copy()


class OrcOptions(C.Structure):  # mh_options, include/mh_kernel.h
    _fields_ = [("seed", C.c_uint64), ("track_best", C.c_int32), ("rng", C.c_int32),
                ("n_temps", C.c_int32), ("swap_interval", C.c_int32), ("beta_min", C.c_double),
                ("reserved", C.c_int32 * 4)]


def run_chains(room, chains: int, iterations: int, seed: int, chain_begin: int = 0,
               threads: int = 1, state: bool = False, track: int = 0, rng: int = 0,
               temps: int = 1, swap_interval: int = 1, beta_min: float = 2.0):
    """Runs the restated chain loop. Returns (points [chains,N,6] float32 or state
    [chains,N,6] float64 (x,y,z,rotX,rotY,rotZ), costs [chains,8] float32, accepted [chains]
    int64). `track` = 1 / 2 returns each chain's lowest / highest-total configuration instead
    of its final one (the reference's commented-out cfgBest, Kernel.cu:779-816). `rng` = 1
    draws from cuRAND's XORWOW seeded as the reference seeds it (mh_options.rng). `temps` > 1
    runs parallel tempering (mh_options.n_temps); outputs are then in rung order per group."""
    lib = load()
    n = room.n
    cs = (C.c_float * (8 * chains))()
    acc = (C.c_int64 * chains)()
    if track or rng or temps > 1:
        state = True
        buf = (C.c_uint8 * (72 * n * chains))()
        opts = OrcOptions(seed, track, rng, temps, swap_interval, beta_min)
        rc = lib.orc_run_chains_ex(C.byref(orc_room(room)), C.cast(room.cfg, C.c_void_p),
                                   C.byref(opts), chain_begin, chains, iterations, threads,
                                   C.cast(buf, C.c_void_p), C.cast(cs, C.c_void_p), acc)
    elif state:
        from numpy.lib import recfunctions  # noqa: F401
        buf = (C.c_uint8 * (72 * n * chains))()
        rc = lib.orc_run_chains_state(C.byref(orc_room(room)), C.cast(room.cfg, C.c_void_p), seed,
                                      chain_begin, chains, iterations, threads,
                                      C.cast(buf, C.c_void_p), C.cast(cs, C.c_void_p), acc)
    else:
        buf = (C.c_float * (6 * n * chains))()
        rc = lib.orc_run_chains(C.byref(orc_room(room)), C.cast(room.cfg, C.c_void_p), seed,
                                chain_begin, chains, iterations, threads,
                                C.cast(buf, C.c_void_p), C.cast(cs, C.c_void_p), acc)
    if rc != 0:
        raise RuntimeError(lib.orc_last_error().decode())
    c8 = np.frombuffer(bytes(cs), dtype=np.float32).reshape(chains, 8).copy()
    a = np.frombuffer(bytes(acc), dtype=np.int64).copy()
    if state:
        raw = np.frombuffer(bytes(buf), dtype=np.uint8).reshape(chains, n, 72)
        d = np.zeros((chains, n, 6), dtype=np.float64)
        for k in range(6):
            d[:, :, k] = raw[:, :, 8 * k:8 * k + 8].copy().view(np.float64)[:, :, 0]
        return d, c8, a
    return np.frombuffer(bytes(buf), dtype=np.float32).reshape(chains, n, 6).copy(), c8, a


def u1_uphill_draws(reset: bool = False) -> int:
    """Accept draws of u == 1.0f against an uphill proposal (threshold exactly 1, so Accept
    rejects, Kernel.cu:706-713) that the oracle's chains have seen."""
    return int(load().orc_u1_uphill_draws(1 if reset else 0))


def set_step_offlimits(on: bool) -> None:
    """OffLimits in every step's Costs() (True, the reference's loop Kernel.cu:785-828) or only
    for the output configurations (False: the same outputs bit for bit, faster; OffLimits never
    enters totalCosts, :547). Process-wide."""
    load().orc_set_step_offlimits(1 if on else 0)


def index_n_draws(reset: bool = False) -> int:
    """Draws of index nObjs (u == 1.0f, Kernel.cu:566-574) the oracle's picks have seen."""
    return int(load().orc_index_n_draws(1 if reset else 0))


def rng_init(seed: int, subsequence: int, kind: int = PHILOX) -> OrcRng:
    lib = load()
    r = OrcRng()
    if kind == PHILOX:
        lib.orc_rng_init(C.byref(r), seed, subsequence)
    else:
        lib.orc_rng_init_xorwow(C.byref(r), seed, subsequence, kind)
    return r


def rng_streams(seed: int, subsequence: int, n: int, kind: int = PHILOX):
    """(u32, uniform, normal) streams, each restarted at draw 0 (as mh_debug_rng_ex)."""
    lib = load()
    r = rng_init(seed, subsequence, kind)
    u = np.array([lib.orc_rng_next(C.byref(r)) for _ in range(n)], dtype=np.uint32)
    r = rng_init(seed, subsequence, kind)
    f = np.array([lib.orc_rng_uniform(C.byref(r)) for _ in range(n)], dtype=np.float32)
    r = rng_init(seed, subsequence, kind)
    g = np.array([lib.orc_rng_normal(C.byref(r)) for _ in range(n)], dtype=np.float32)
    return u, f, g


# mh_math.h's numerics probes (MH_PROBE_*), in order
PROBES = ["bm_log", "bm_sincos", "cos_f32", "xw_log", "xw_sincos", "atan2_room", "atan2_bits",
          "atan2f_room", "atan2f_bits", "exp_accept", "exp_any", "accept"]


def probe_width(fn: int) -> int:
    return 2 if PROBES[fn] in ("bm_sincos", "xw_sincos") else 1


def math_eval(fn: int, start: int, count: int, threads: int = 8, libm: bool = False) -> np.ndarray:
    """mh_math.h's probe `fn` (or the C library's, libm=True) at argument indices start ..
    start + count - 1: float64 [count, width]."""
    lib = load()
    out = np.empty((count, probe_width(fn)), dtype=np.float64)
    f = lib.orc_math_eval_libm if libm else lib.orc_math_eval
    if f(fn, start, count, threads, out.ctypes.data) != 0:
        raise RuntimeError(lib.orc_last_error().decode())
    return out


MATH_FUNCTIONS = {"log": 0, "exp": 1, "sin": 2, "cos": 3, "atan2": 4, "sin_medium": 5}


def math_apply(name: str, a, b=None) -> np.ndarray:
    """mh_math.h's `name` on float64 arguments a (and b for atan2(a, b))."""
    lib = load()
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = None if b is None else np.ascontiguousarray(b, dtype=np.float64)
    out = np.empty_like(a)
    if lib.orc_math_apply(MATH_FUNCTIONS[name], a.ctypes.data, None if b is None else b.ctypes.data,
                          len(a), out.ctypes.data) != 0:
        raise RuntimeError(lib.orc_last_error().decode())
    return out
