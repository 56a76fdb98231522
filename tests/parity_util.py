"""Shared checks of the GPU parity tests: chain-by-chain bit identity with the oracle, with the
exact fork count in every failure message and in a warning that survives `pytest -q`."""
import warnings

import numpy as np

REL_TOL = 1e-4  # BASELINE.json north_star: "within 1e-4 relative fp32"


class ParityReport(UserWarning):
    """One line per parity check: how many chains were compared and how many forked."""


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a.view(np.uint64)


def forked_chains(pts, costs, ref_pts, ref_costs):
    """Indices of chains whose final points or costs differ from the oracle's in any bit."""
    ref_pts = np.asarray(ref_pts)
    if ref_pts.dtype == np.float64:  # oracle state -> the float points the device reports
        ref_pts = ref_pts.astype(np.float32)
    same = np.all(bits(pts) == bits(ref_pts), axis=tuple(range(1, np.ndim(pts)))) & np.all(
        bits(costs) == bits(ref_costs), axis=1)
    return np.flatnonzero(~same)


def check_chains(name, pts, costs, ref_pts, ref_costs, ids=None, report=False):
    """Asserts every chain bit-identical to the oracle and the mean final total within REL_TOL.
    `ids` maps row k to its global chain id (for the message). With `report`, the counts are
    also emitted as a ParityReport warning."""
    forked = forked_chains(pts, costs, ref_pts, ref_costs)
    ids = np.arange(len(costs)) if ids is None else np.asarray(ids)
    got_mean = float(np.asarray(costs)[:, 0].astype(np.float64).mean())
    ref_mean = float(np.asarray(ref_costs)[:, 0].astype(np.float64).mean())
    rel = abs(got_mean - ref_mean) / max(abs(ref_mean), 1e-6)
    msg = (f"{name}: {len(forked)} of {len(costs)} chains forked"
           + (f" (global ids {ids[forked][:32].tolist()})" if len(forked) else "")
           + f"; mean final total {got_mean:.9g} vs oracle {ref_mean:.9g} (rel {rel:.3g})")
    print(msg)
    if report:
        warnings.warn(msg, ParityReport)
    assert len(forked) == 0, msg
    assert rel <= REL_TOL, msg
    return msg
