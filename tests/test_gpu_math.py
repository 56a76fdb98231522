"""Device vs oracle numerics, exhaustively: the project's transcendentals (mh_math.h) compiled by
hipcc for gfx950 (mh_debug_math, the device code the chains run) and by gcc for the oracle
(orc_math_eval) return the same bits.

Every transcendental the chain uses is one of these probes:
- Box-Muller (the Philox normals, Kernel.cu:605,608,641 stand-in): log(a 2^-32 + 2^-33) and
  sincos(2 pi (b 2^-32 + 2^-33)) over all 2^32 a and b. The normal is sqrt(-2 log) times sin or
  cos, each operation correctly rounded, so these two exhaustive checks cover every normal.
- cosf in FocalPointCosts (:277): all 2^32 float bit patterns.
- cuRAND's Box-Muller (the XORWOW stream): logf(u) and sincos(v) over all 2^32 x and y.
- atan2 in theta (:173), atan2f in phi (:187) and exp in Accept (:712): 2^30 sampled arguments
  each, from the distributions the chains produce (float differences of room coordinates; BETA
  (star - cur) around totals of up to 2^15) and from all float bit patterns.
- Accept's decision itself (:712): the device decides most draws with an fp32 exp screen
  (mh_common.h accept_u) and must return the exact decision; 2^30 (u, x) pairs, three in four
  within 1e-4 of the threshold.
A mismatch count is reported for each (MathReport warnings); the bar is zero.
"""
import os
import warnings

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHUNK = 1 << 26
THREADS = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)


class MathReport(UserWarning):
    pass


def _compare(mh, orc, fn, start, count):
    """(mismatches, first mismatching index or None) of probe fn over [start, start + count)."""
    width = orc.probe_width(fn)
    bad, first = 0, None
    for s in range(start, start + count, CHUNK):
        n = min(CHUNK, start + count - s)
        dev = mh.debug_math(fn, s, n, width)
        ref = orc.math_eval(fn, s, n, threads=THREADS)
        diff = dev.view(np.uint64) != ref.view(np.uint64)
        diff &= ~(np.isnan(dev) & np.isnan(ref))  # (NaN payloads are not compared)
        rows = diff.any(axis=1)
        k = int(rows.sum())
        if k and first is None:
            first = s + int(np.argmax(rows))
        bad += k
        del dev, ref, diff, rows
    return bad, first


def _report(orc, fn, count, bad, first):
    msg = (f"MathReport probe {orc.PROBES[fn]}: {count} arguments, device vs oracle mismatches "
           f"{bad}" + (f" (first at argument {first})" if first is not None else ""))
    warnings.warn(msg, MathReport)
    return msg


EXHAUSTIVE = ["bm_log", "bm_sincos", "cos_f32", "xw_log", "xw_sincos"]


@pytest.mark.parametrize("quarter", range(4))
@pytest.mark.parametrize("probe", EXHAUSTIVE)
def test_exhaustive_32bit_domain(mh, orc, hiplib, probe, quarter):
    fn = orc.PROBES.index(probe)
    start, count = quarter << 30, 1 << 30
    bad, first = _compare(mh, orc, fn, start, count)
    msg = _report(orc, fn, count, bad, first)
    assert bad == 0, msg


SAMPLED = ["atan2_room", "atan2_bits", "atan2f_room", "atan2f_bits", "exp_accept", "exp_any",
           "accept"]  # (accept: the device's fp32-screened decision against the exact one)


@pytest.mark.parametrize("probe", SAMPLED)
def test_sampled_arguments(mh, orc, hiplib, probe):
    fn = orc.PROBES.index(probe)
    count = 1 << 30
    bad, first = _compare(mh, orc, fn, 0, count)
    msg = _report(orc, fn, count, bad, first)
    assert bad == 0, msg


def test_probe_edges(mh, orc, hiplib):
    """The ends of each 32-bit domain (zero, the largest draw, infinities and NaN bit patterns of
    cosf) and the start of every sampled stream, elementwise."""
    for fn in range(len(orc.PROBES)):
        for start in (0, (1 << 32) - 4096, 0x7F7FF000, 0x7F800000 - 8, 0xFF800000 - 8):
            dev = mh.debug_math(fn, start, 4096, orc.probe_width(fn))
            ref = orc.math_eval(fn, start, 4096, threads=4)
            same = (dev.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(dev) & np.isnan(ref))
            assert same.all(), (orc.PROBES[fn], start, int(np.argmin(same.all(axis=1))))
