"""Rooms the sampler is exercised on.

* main_fixture(): the console harness's hard-coded room, KernelFolder/Kernel/Kernel.cu:1007-1194
  (N = 32 objects at (2i, 2i), two clearances, one relationship). WeightOffLimits is left
  uninitialised there; it is 0 here.
* synthetic_room(n): the deterministic synthetic room of SURVEY.md 8(d) used for the benchmark
  configurations (N = 8, 64, 256): square room W = H = 2.5*sqrt(N), C = N/4 clearances,
  R = N/2 relationships, splitmix64(0x5EED0000 + N) for every random quantity.
"""
from __future__ import annotations

import ctypes as C
import math

from .abi import (Room, Surface, positionAndRotation, rectangle, relationshipAngleStruct,
                  relationshipStruct, vertex)

PI = 3.1416  # Kernel.cu:31


def _verts(pts):
    arr = (vertex * len(pts))()
    for i, (x, y) in enumerate(pts):
        arr[i] = vertex(x, y, 0.0)
    return arr


def main_fixture() -> Room:
    """Kernel.cu:1007-1166 (the room main() passes to KernelWrapper at :1198)."""
    n, nrel, ncl = 32, 1, 2
    srf = Surface()
    srf.nObjs, srf.nRelationships, srf.nClearances = n, nrel, ncl
    srf.WeightFocalPoint = -2.0
    srf.WeightPairWise = -2.0
    srf.WeightVisualBalance = 1.5
    srf.WeightSymmetry = -2.0
    srf.WeightOffLimits = 0.0  # uninitialised in main(); 0 as in SURVEY.md 8(c)
    srf.WeightClearance = -2.0
    srf.WeightSurfaceArea = -2.0
    srf.centroidX = srf.centroidY = 0.0
    srf.focalX = srf.focalY = 5.0
    srf.focalRot = 0.0
    surface = _verts([(10, 10), (10, 0), (0, 0), (0, 10)])
    # 16 vertices: two clearance shapes then two off-limits shapes (Kernel.cu:1044-1109). The
    # reference copies 4*(C+N) = 136 vertices from this 16-entry array (an over-read,
    # Kernel.cu:906); this library reads only the vertices a rectangle indexes.
    vtx = _verts([(2, 2), (2, 0), (0, 0), (0, 2),
                  (3, 2), (3, 0), (1, 0), (1, 2),
                  (2, 2), (2, 0), (0, 0), (0, 2),
                  (3, 2), (3, 0), (1, 0), (1, 2)])
    clearances = (rectangle * ncl)(rectangle(0, 1, 2, 3, 0), rectangle(4, 5, 6, 7, 1))
    offlimits = (rectangle * n)()
    for i in range(n):
        offlimits[i] = rectangle(8, 9, 10, 11, 0) if i % 2 == 0 else rectangle(12, 13, 14, 15, 1)
    cfg = (positionAndRotation * n)()
    for i in range(n):
        cfg[i] = positionAndRotation(i * 2.0, i * 2.0, 0.0, 0.0, 0.0, 0.0, False, 1.0, 1.0)
    rss = (relationshipStruct * nrel)()
    rss[0].TargetRange.targetRangeStart = 2.0
    rss[0].TargetRange.targetRangeEnd = 4.0
    rss[0].DegreesOfAtrraction = 2.0
    rss[0].SourceIndex, rss[0].TargetIndex = 0, 1
    rsa = (relationshipAngleStruct * nrel)()
    rsa[0].angleMin = PI / 4
    rsa[0].angleMax = 5 * PI / 8
    rsa[0].SourceIndex, rsa[0].TargetIndex = 0, 1
    return Room(srf, cfg, rss, rsa, clearances, offlimits, vtx, surface, name="main_fixture")


class SplitMix64:
    """splitmix64 (Steele, Lea, Flood 2014)."""

    MASK = (1 << 64) - 1

    def __init__(self, seed: int):
        self.s = seed & self.MASK

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & self.MASK
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & self.MASK
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & self.MASK
        return z ^ (z >> 31)

    def uniform(self, lo: float, hi: float) -> float:
        u = (self.next() >> 11) * (1.0 / 9007199254740992.0)  # [0, 1)
        return lo + (hi - lo) * u

    def below(self, k: int) -> int:
        return self.next() % k


def synthetic_room(n: int, freeze_every: int = 0, seed: int | None = None,
                   n_rel: int | None = None) -> Room:
    """SURVEY.md 8(d) synthetic room. Draw order: per clearance (a, b, source); per object
    (a, b, x, y, rotY); per relationship (source, target != source). `n_rel` overrides the
    N/2 relationships (test rooms with more relationships than objects)."""
    if n < 1:
        raise ValueError("n >= 1")
    rng = SplitMix64(0x5EED0000 + n if seed is None else seed)
    w = 2.5 * math.sqrt(n)
    ncl = n // 4
    nrel = (n // 2 if n >= 2 else 0) if n_rel is None else (n_rel if n >= 2 else 0)
    srf = Surface()
    srf.nObjs, srf.nRelationships, srf.nClearances = n, nrel, ncl
    srf.WeightFocalPoint = 2.0
    srf.WeightPairWise = 2.0
    srf.WeightVisualBalance = 1.5
    srf.WeightSymmetry = 2.0
    srf.WeightOffLimits = 2.0
    srf.WeightClearance = 2.0
    srf.WeightSurfaceArea = 2.0
    srf.centroidX = srf.centroidY = w
    srf.focalX, srf.focalY = w / 2, w
    srf.focalRot = PI / 2
    surface = _verts([(w, w), (w, 0), (0, 0), (0, w)])
    verts = []
    clearances = (rectangle * max(ncl, 1))()
    for i in range(ncl):
        a, b = rng.uniform(0.5, 2.0), rng.uniform(0.5, 2.0)
        src = rng.below(n)
        base = len(verts)
        verts += [(a, b), (a, 0.0), (0.0, 0.0), (0.0, b)]
        clearances[i] = rectangle(base, base + 1, base + 2, base + 3, src)
    offlimits = (rectangle * n)()
    cfg = (positionAndRotation * n)()
    for j in range(n):
        a, b = rng.uniform(0.5, 2.0), rng.uniform(0.5, 2.0)
        x, y = rng.uniform(0.0, w), rng.uniform(0.0, w)
        rot = rng.uniform(0.0, 2 * PI)
        base = len(verts)
        verts += [(a, b), (a, 0.0), (0.0, 0.0), (0.0, b)]
        offlimits[j] = rectangle(base, base + 1, base + 2, base + 3, j)
        frozen = bool(freeze_every) and (j % freeze_every == freeze_every - 1)
        cfg[j] = positionAndRotation(x, y, 0.0, 0.0, rot, 0.0, frozen, a, b)
    rss = (relationshipStruct * max(nrel, 1))()
    rsa = (relationshipAngleStruct * max(nrel, 1))()
    for k in range(nrel):
        s = rng.below(n)
        t = rng.below(n - 1)
        t = t + 1 if t >= s else t
        rss[k].TargetRange.targetRangeStart = 1.0
        rss[k].TargetRange.targetRangeEnd = 3.0
        rss[k].DegreesOfAtrraction = 1.0
        rss[k].SourceIndex, rss[k].TargetIndex = s, t
        rsa[k].angleMin = PI / 4
        rsa[k].angleMax = 5 * PI / 8
        rsa[k].SourceIndex, rsa[k].TargetIndex = s, t
    vtx = _verts(verts)
    return Room(srf, cfg, rss, rsa, clearances, offlimits, vtx, surface, name=f"synthetic{n}")


def clone_cfg(room: Room):
    arr = (positionAndRotation * room.n)()
    C.memmove(arr, room.cfg, C.sizeof(arr))
    return arr
