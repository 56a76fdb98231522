"""ctypes mirror of the C ABI in include/mh_kernel.h (the reference's KernelWrapper surface,
KernelFolder/Kernel/Kernel.cu:43-149 structs and :873 export).

This is the binding a Python caller (tests, bench.py) uses; the C# host of the reference binds
the same symbols with P/Invoke. The library is the HIP build in this package
directory; there is no CPU fallback: every compute entry point raises if libmhgpu.so is absent.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "libmhgpu.so"


# ---- wire structs (Kernel.cu:43-149) ---------------------------------------------------------

class vertex(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("z", C.c_double)]


class rectangle(C.Structure):
    _fields_ = [("point1Index", C.c_int), ("point2Index", C.c_int), ("point3Index", C.c_int),
                ("point4Index", C.c_int), ("SourceIndex", C.c_int)]


class positionAndRotation(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("z", C.c_double),
                ("rotX", C.c_double), ("rotY", C.c_double), ("rotZ", C.c_double),
                ("frozen", C.c_bool), ("length", C.c_double), ("width", C.c_double)]


class targetRangeStruct(C.Structure):
    _fields_ = [("targetRangeStart", C.c_double), ("targetRangeEnd", C.c_double)]


class relationshipStruct(C.Structure):
    _fields_ = [("TargetRange", targetRangeStruct), ("SourceIndex", C.c_int),
                ("TargetIndex", C.c_int), ("DegreesOfAtrraction", C.c_double)]


class relationshipAngleStruct(C.Structure):
    _fields_ = [("angleMin", C.c_double), ("angleMax", C.c_double),
                ("SourceIndex", C.c_int), ("TargetIndex", C.c_int)]


class Surface(C.Structure):
    _fields_ = [("nObjs", C.c_int), ("nRelationships", C.c_int), ("nClearances", C.c_int),
                ("WeightFocalPoint", C.c_float), ("WeightPairWise", C.c_float),
                ("WeightVisualBalance", C.c_float), ("WeightSymmetry", C.c_float),
                ("WeightOffLimits", C.c_float), ("WeightClearance", C.c_float),
                ("WeightSurfaceArea", C.c_float),
                ("centroidX", C.c_double), ("centroidY", C.c_double),
                ("focalX", C.c_double), ("focalY", C.c_double), ("focalRot", C.c_double)]


class gpuConfig(C.Structure):
    _fields_ = [("gridxDim", C.c_int), ("gridyDim", C.c_int), ("blockxDim", C.c_int),
                ("blockyDim", C.c_int), ("blockzDim", C.c_int), ("iterations", C.c_int)]


class point(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float),
                ("rotX", C.c_float), ("rotY", C.c_float), ("rotZ", C.c_float)]


class resultCosts(C.Structure):
    _fields_ = [("totalCosts", C.c_float), ("PairWiseCosts", C.c_float),
                ("VisualBalanceCosts", C.c_float), ("FocalPointCosts", C.c_float),
                ("SymmetryCosts", C.c_float), ("ClearanceCosts", C.c_float),
                ("OffLimitsCosts", C.c_float), ("SurfaceAreaCosts", C.c_float)]


class result(C.Structure):
    _fields_ = [("points", C.POINTER(point)), ("costs", resultCosts)]


class mh_summary(C.Structure):
    _fields_ = [("sum_total", C.c_double), ("best_total", C.c_float), ("pad", C.c_int32),
                ("best_chain", C.c_int64), ("n_chains", C.c_int64), ("accepted", C.c_int64)]


class mh_options(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("track_best", C.c_int32), ("rng", C.c_int32),
                ("n_temps", C.c_int32), ("swap_interval", C.c_int32), ("beta_min", C.c_double),
                ("reserved", C.c_int32 * 4)]


def options(seed: int, track: int = 0, rng: int = 0, temps: int = 1, swap_interval: int = 1,
            beta_min: float = 2.0) -> "mh_options":
    return mh_options(seed, track, rng, temps, swap_interval, beta_min)


MH_TRACK_OFF, MH_TRACK_LOWEST, MH_TRACK_HIGHEST = 0, 1, 2
MH_RNG_PHILOX, MH_RNG_CURAND_XORWOW = 0, 1

STRUCT_LAYOUT = {  # (size, {field: offset}) as static_assert-ed in include/mh_kernel.h
    vertex: (24, {}),
    rectangle: (20, {}),
    positionAndRotation: (72, {"rotZ": 40, "frozen": 48, "length": 56, "width": 64}),
    targetRangeStruct: (16, {}),
    relationshipStruct: (32, {"SourceIndex": 16, "TargetIndex": 20, "DegreesOfAtrraction": 24}),
    relationshipAngleStruct: (24, {"SourceIndex": 16}),
    Surface: (80, {"WeightFocalPoint": 12, "WeightSurfaceArea": 36, "centroidX": 40,
                   "focalRot": 72}),
    gpuConfig: (24, {}),
    point: (24, {}),
    resultCosts: (32, {}),
    result: (40, {"costs": 8}),
    mh_summary: (40, {}),
    mh_options: (48, {"track_best": 8, "rng": 12, "n_temps": 16, "swap_interval": 20,
                      "beta_min": 24}),
}

COST_FIELDS = ["totalCosts", "PairWiseCosts", "VisualBalanceCosts", "FocalPointCosts",
               "SymmetryCosts", "ClearanceCosts", "OffLimitsCosts", "SurfaceAreaCosts"]

# Every symbol include/mh_kernel.h declares.
EXPORTS = ["KernelWrapper", "KernelWrapperSeeded", "KernelWrapperEx", "KernelFreeResult",
           "KernelReleaseCache", "KernelLastError", "KernelEvaluateCosts", "mh_session_create", "mh_session_create_ex",
           "mh_session_run", "mh_session_finalize",
           "mh_session_download", "mh_session_current_costs", "mh_session_summary",
           "mh_session_geometry", "mh_session_occupancy",
           "mh_session_destroy", "mh_debug_rng", "mh_debug_rng_ex", "mh_debug_collectives",
           "mh_debug_math", "mh_debug_wrapper_step"]

P = C.POINTER


class MHError(RuntimeError):
    pass


_lib = None


def _check_build_matches_sources(p: Path) -> None:
    """The product library must have been built from the sources beside it: build() records
    their hash (libmhgpu.so.srchash); a library built from other sources is refused."""
    stamp = p.with_name(p.name + ".srchash")
    entry = p.parents[1] / "__graft_entry__.py"
    if not entry.exists():  # an installed copy without the tree: nothing to compare against
        return
    import importlib.util
    spec = importlib.util.spec_from_file_location("_mh_graft_entry", entry)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    want = mod.source_hash(("-DMH_CHECK=1",) if p.name == "libmhgpu_check.so" else ())
    got = stamp.read_text().strip() if stamp.exists() else "(no record)"
    if got != want:
        raise MHError(f"{p} was not built from the sources in this tree (recorded {got[:12]}, "
                      f"tree {want[:12]}): run __graft_entry__.build()")


def load_library(path: os.PathLike | str | None = None) -> C.CDLL:
    """Loads libmhgpu.so (built by __graft_entry__.build()). Raises if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else Path(os.environ.get("MH_LIB", LIB_PATH))
    if not p.exists():
        raise MHError(f"{p} not found: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    if p.resolve() in (LIB_PATH.resolve(), LIB_PATH.with_name("libmhgpu_check.so").resolve()):
        _check_build_matches_sources(p)
    lib = C.CDLL(str(p))
    room_args = [P(relationshipStruct), P(relationshipAngleStruct), P(positionAndRotation),
                 P(rectangle), P(rectangle), P(vertex), P(vertex), P(Surface)]
    lib.KernelWrapper.argtypes = room_args + [P(gpuConfig)]
    lib.KernelWrapper.restype = P(result)
    lib.KernelWrapperSeeded.argtypes = room_args + [P(gpuConfig), C.c_uint64]
    lib.KernelWrapperSeeded.restype = P(result)
    lib.KernelWrapperEx.argtypes = room_args + [P(gpuConfig), P(mh_options)]
    lib.KernelWrapperEx.restype = P(result)
    lib.KernelFreeResult.argtypes = [P(result)]
    lib.KernelFreeResult.restype = None
    if hasattr(lib, "KernelReleaseCache"):  # (A/B variants of earlier revisions lack it)
        lib.KernelReleaseCache.argtypes = []
        lib.KernelReleaseCache.restype = C.c_int
    lib.KernelLastError.argtypes = []
    lib.KernelLastError.restype = C.c_char_p
    lib.KernelEvaluateCosts.argtypes = [P(relationshipStruct), P(relationshipAngleStruct),
                                        P(positionAndRotation), C.c_int, P(rectangle),
                                        P(rectangle), P(vertex), P(vertex), P(Surface),
                                        P(resultCosts)]
    lib.KernelEvaluateCosts.restype = C.c_int
    lib.mh_session_create.argtypes = room_args + [C.c_int, C.c_int64, C.c_int64, C.c_uint64]
    lib.mh_session_create.restype = C.c_void_p
    lib.mh_session_create_ex.argtypes = room_args + [C.c_int, C.c_int64, C.c_int64, P(mh_options)]
    lib.mh_session_create_ex.restype = C.c_void_p
    lib.mh_session_run.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    lib.mh_session_run.restype = C.c_int
    lib.mh_session_finalize.argtypes = [C.c_void_p, C.c_void_p]
    lib.mh_session_finalize.restype = C.c_int
    lib.mh_session_download.argtypes = [C.c_void_p, P(point), P(resultCosts)]
    lib.mh_session_download.restype = C.c_int
    lib.mh_session_current_costs.argtypes = [C.c_void_p, P(resultCosts)]
    lib.mh_session_current_costs.restype = C.c_int
    lib.mh_session_summary.argtypes = [C.c_void_p, P(mh_summary)]
    lib.mh_session_summary.restype = C.c_int
    lib.mh_session_geometry.argtypes = [C.c_void_p, P(C.c_int), P(C.c_int), P(C.c_int)]
    lib.mh_session_geometry.restype = C.c_int
    lib.mh_session_occupancy.argtypes = [C.c_void_p, P(C.c_int)]
    lib.mh_session_occupancy.restype = C.c_int
    lib.mh_session_destroy.argtypes = [C.c_void_p]
    lib.mh_session_destroy.restype = None
    if hasattr(lib, "mh_debug_wrapper_step"):  # (A/B variants of earlier revisions lack it)
        lib.mh_debug_wrapper_step.argtypes = [P(C.c_int), P(C.c_int)]
        lib.mh_debug_wrapper_step.restype = C.c_int
    lib.mh_debug_collectives.argtypes = [C.c_int, P(C.c_float), P(C.c_int), P(C.c_int)]
    lib.mh_debug_collectives.restype = C.c_int
    lib.mh_debug_rng.argtypes = [C.c_uint64, C.c_uint64, C.c_int, P(C.c_uint32), P(C.c_float),
                                 P(C.c_float)]
    lib.mh_debug_rng.restype = C.c_int
    lib.mh_debug_rng_ex.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_int, P(C.c_uint32),
                                    P(C.c_float), P(C.c_float)]
    lib.mh_debug_rng_ex.restype = C.c_int
    if hasattr(lib, "mh_debug_math"):  # (A/B variants of earlier revisions lack it)
        lib.mh_debug_math.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_void_p]
        lib.mh_debug_math.restype = C.c_int
    if path is None:
        _lib = lib
    return lib


def last_error(lib: C.CDLL | None = None) -> str:
    lib = lib or load_library()
    return (lib.KernelLastError() or b"").decode()


# ---- room container ------------------------------------------------------------------------

class Room:
    """The eight KernelWrapper inputs that describe a room, as ctypes arrays (the exact bytes a
    P/Invoke caller passes)."""

    def __init__(self, srf: Surface, cfg, rss, rsa, clearances, offlimits, vertices,
                 surface_rectangle, name: str = "room"):
        self.name = name
        self.srf = srf
        self.cfg = cfg
        self.rss = rss
        self.rsa = rsa
        self.clearances = clearances
        self.offlimits = offlimits
        self.vertices = vertices
        self.surface_rectangle = surface_rectangle

    @property
    def n(self) -> int:
        return self.srf.nObjs

    def args(self, cfg=None):
        c = self.cfg if cfg is None else cfg
        return (self.rss, self.rsa, c, self.clearances, self.offlimits, self.vertices,
                self.surface_rectangle, C.byref(self.srf))

    def cfg_array(self) -> np.ndarray:
        """cfg as a structured numpy view (x, y, z, rotX, rotY, rotZ, frozen, length, width)."""
        return np.ctypeslib.as_array(self.cfg).copy()


def costs_to_array(cs) -> np.ndarray:
    """resultCosts array -> float32 [n, 8] in resultCosts field order."""
    a = np.ctypeslib.as_array(cs) if not isinstance(cs, np.ndarray) else cs
    return np.frombuffer(bytes(memoryview(a)), dtype=np.float32).reshape(-1, 8).copy()


def points_to_array(pts, count: int) -> np.ndarray:
    buf = (point * count).from_address(C.addressof(pts.contents)) if hasattr(pts, "contents") else pts
    return np.frombuffer(bytes(memoryview(buf)), dtype=np.float32).reshape(count, 6).copy()


# ---- calls -----------------------------------------------------------------------------------

def kernel_wrapper(room: Room, chains: int, iterations: int, seed: int | None = None,
                   block_x: int = 64, track: int = MH_TRACK_OFF, rng: int = MH_RNG_PHILOX,
                   temps: int = 1, swap_interval: int = 1, beta_min: float = 2.0):
    """Calls KernelWrapper (or KernelWrapperSeeded, or KernelWrapperEx when `track` or `rng`
    is set) exactly as the reference's caller does and returns (points [chains, N, 6] float32,
    costs [chains, 8] float32)."""
    lib = load_library()
    g = gpuConfig(chains, 0, block_x, 0, 0, iterations)
    if track or rng or temps > 1:
        if seed is None:
            raise ValueError("KernelWrapperEx needs an explicit seed")
        opts = options(seed, track, rng, temps, swap_interval, beta_min)
        res = lib.KernelWrapperEx(*room.args(), C.byref(g), C.byref(opts))
    elif seed is None:
        res = lib.KernelWrapper(*room.args(), C.byref(g))
    else:
        res = lib.KernelWrapperSeeded(*room.args(), C.byref(g), C.c_uint64(seed))
    if not res:
        raise MHError(last_error(lib))
    try:
        n = room.n
        pts = (point * (chains * n)).from_address(C.cast(res[0].points, C.c_void_p).value)
        p = np.frombuffer(bytes(memoryview(pts)), dtype=np.float32).reshape(chains, n, 6).copy()
        rs = (result * chains).from_address(C.cast(res, C.c_void_p).value)
        costs = np.array([[getattr(rs[i].costs, f) for f in COST_FIELDS] for i in range(chains)],
                         dtype=np.float32)
        # every result[i].points must point into the one block, at i * N (Kernel.cu:981)
        base = C.cast(res[0].points, C.c_void_p).value
        for i in (0, chains - 1):
            assert C.cast(rs[i].points, C.c_void_p).value == base + i * n * C.sizeof(point)
    finally:
        lib.KernelFreeResult(res)
    return p, costs


STEP_KINDS = {0: "full", 1: "incremental", 2: "full-few", 3: "speculative"}


HIP_ATTR_MULTIPROCESSOR_COUNT = 63  # hipDeviceAttributeMultiprocessorCount (ROCm 7.2 headers)


def device_cus(device: int = 0) -> int:
    """Compute units of a HIP device, asked of the HIP runtime libmhgpu.so uses (not torch's:
    a test process that has already initialised that runtime must not initialise a second)."""
    load_library()
    hip = C.CDLL("libamdhip64.so.7")
    v = C.c_int()
    if hip.hipDeviceGetAttribute(C.byref(v), HIP_ATTR_MULTIPROCESSOR_COUNT, device) != 0:
        raise MHError("hipDeviceGetAttribute failed")
    return v.value


def wrapper_step_kernel():
    """(lanes per chain, kind) of the step kernel this thread's last kernel_wrapper call ran."""
    lib = load_library()
    lanes, kind = C.c_int(), C.c_int()
    if lib.mh_debug_wrapper_step(C.byref(lanes), C.byref(kind)) != 0:
        raise MHError("no KernelWrapper call on this thread yet")
    return lanes.value, STEP_KINDS[kind.value]


def release_cache() -> int:
    """KernelReleaseCache(): frees KernelWrapper's idle pooled sessions; returns how many."""
    return int(load_library().KernelReleaseCache())


def evaluate_costs(room: Room, cfgs) -> np.ndarray:
    """KernelEvaluateCosts on a ctypes array of len(cfgs) == k * N configurations."""
    lib = load_library()
    k = len(cfgs) // room.n
    out = (resultCosts * max(k, 1))()
    rc = lib.KernelEvaluateCosts(room.rss, room.rsa, cfgs, k, room.clearances, room.offlimits,
                                 room.vertices, room.surface_rectangle, C.byref(room.srf), out)
    if rc != 0:
        raise MHError(last_error(lib))
    return costs_to_array(out)[:k]


def debug_rng(seed: int, subsequence: int, n: int, rng: int = MH_RNG_PHILOX):
    lib = load_library()
    u = (C.c_uint32 * n)()
    f = (C.c_float * n)()
    g = (C.c_float * n)()
    if lib.mh_debug_rng_ex(rng, C.c_uint64(seed), C.c_uint64(subsequence), n, u, f, g) != 0:
        raise MHError(last_error(lib))
    return (np.frombuffer(bytes(u), dtype=np.uint32).copy(),
            np.frombuffer(bytes(f), dtype=np.float32).copy(),
            np.frombuffer(bytes(g), dtype=np.float32).copy())


# doubles each probe writes per argument (mh_math.h mh_probe_width: the sincos probes 2)
MH_PROBE_COUNT = 12
_PROBE_WIDTH = {1: 2, 4: 2}  # MH_PROBE_BM_SINCOS, MH_PROBE_XW_SINCOS


def probe_width(fn: int) -> int:
    return _PROBE_WIDTH.get(fn, 1)


def debug_math(fn: int, start: int, count: int, width: int | None = None) -> np.ndarray:
    """mh_debug_math: the shared transcendentals' probe `fn` evaluated on the device, float64
    [count, width] (diagnostic; tests/test_gpu_math.py). The C side writes probe_width(fn)
    doubles per argument, so the buffer is sized from `fn`; a `width` that disagrees is an
    error, not a short buffer."""
    if not 0 <= fn < MH_PROBE_COUNT:
        raise ValueError(f"unknown probe {fn}")
    if width is not None and width != probe_width(fn):
        raise ValueError(f"probe {fn} writes {probe_width(fn)} values per argument, not {width}")
    width = probe_width(fn)
    lib = load_library()
    out = np.empty((count, width), dtype=np.float64)
    if lib.mh_debug_math(fn, C.c_uint64(start), C.c_uint64(count), out.ctypes.data) != 0:
        raise MHError(last_error(lib))
    return out


def debug_collectives(L: int, v, iv):
    """The kernels' group collectives over groups of L lanes on 64 lane values (diagnostic)."""
    lib = load_library()
    v = np.ascontiguousarray(v, dtype=np.float32)
    iv = np.ascontiguousarray(iv, dtype=np.int32)
    out = np.zeros(17 * 64, dtype=np.int32)
    if lib.mh_debug_collectives(L, v.ctypes.data_as(P(C.c_float)), iv.ctypes.data_as(P(C.c_int)),
                                out.ctypes.data_as(P(C.c_int))) != 0:
        raise MHError(last_error(lib))
    out = out.reshape(17, 64)
    return {"m1": out[0].view(np.float32), "m2": out[1].view(np.float32), "j1": out[2],
            "max": out[3].view(np.float32), "arg": out[4], "scan": out[5], "total": out[6],
            "imax": out[7], "isum": out[8], "wsum8": out[9:17].view(np.float32)}


class Session:
    """Device-resident chains: the shard one rank owns (chain ids [offset, offset + chains))."""

    def __init__(self, room: Room, chains: int, seed: int, device: int = 0, chain_offset: int = 0,
                 track: int = MH_TRACK_OFF, rng: int = MH_RNG_PHILOX, temps: int = 1,
                 swap_interval: int = 1, beta_min: float = 2.0):
        self.lib = load_library()
        self.room = room
        self.chains = chains
        self.chain_offset = chain_offset
        if track or rng or temps > 1:
            opts = options(seed, track, rng, temps, swap_interval, beta_min)
            h = self.lib.mh_session_create_ex(*room.args(), device, chains, chain_offset,
                                              C.byref(opts))
        else:
            h = self.lib.mh_session_create(*room.args(), device, chains, chain_offset,
                                           C.c_uint64(seed))
        if not h:
            raise MHError(last_error(self.lib))
        self.h = h

    def run(self, iterations: int, stream: int | None = None):
        if self.lib.mh_session_run(self.h, iterations, C.c_void_p(stream or 0)) != 0:
            raise MHError(last_error(self.lib))

    def finalize(self, stream: int | None = None):
        if self.lib.mh_session_finalize(self.h, C.c_void_p(stream or 0)) != 0:
            raise MHError(last_error(self.lib))

    def download(self):
        n = self.room.n
        pts = (point * (self.chains * n))()
        cs = (resultCosts * self.chains)()
        if self.lib.mh_session_download(self.h, pts, cs) != 0:
            raise MHError(last_error(self.lib))
        p = np.frombuffer(bytes(pts), dtype=np.float32).reshape(self.chains, n, 6).copy()
        return p, costs_to_array(cs)

    def current_costs(self) -> np.ndarray:
        """Costs each chain carries for its current state (OffLimits 0), as the accept test saw
        them."""
        cs = (resultCosts * self.chains)()
        if self.lib.mh_session_current_costs(self.h, cs) != 0:
            raise MHError(last_error(self.lib))
        return costs_to_array(cs)

    def summary(self) -> mh_summary:
        s = mh_summary()
        if self.lib.mh_session_summary(self.h, C.byref(s)) != 0:
            raise MHError(last_error(self.lib))
        return s

    def geometry(self):
        """(lanes per chain, chains per workgroup) of the step kernel."""
        return self.step_kernel()[:2]

    def step_kernel(self):
        """(lanes per chain, chains per workgroup, kind) of the step kernel: kind "incremental",
        "full", "full-few" (the full-evaluation instance without the register cap, chosen for
        launches of at most two chains per SIMD) or "speculative" (rooms of at most 8 objects
        with as few chains: mh_spec.hip)."""
        lanes, cpw, inc = C.c_int(), C.c_int(), C.c_int()
        self.lib.mh_session_geometry(self.h, C.byref(lanes), C.byref(cpw), C.byref(inc))
        return lanes.value, cpw.value, STEP_KINDS[inc.value]

    def occupancy(self) -> int:
        """Chains of the step kernel one CU keeps resident (the runtime's occupancy count)."""
        c = C.c_int()
        if self.lib.mh_session_occupancy(self.h, C.byref(c)) != 0:
            raise MHError(last_error(self.lib))
        return c.value

    def close(self):
        if getattr(self, "h", None):
            self.lib.mh_session_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
