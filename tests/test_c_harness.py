"""The reference's console harness as a C program (tests/c/main_room.c restates Kernel.cu:1003-1217):
it compiles as C against include/mh_kernel.h and links libmhgpu.so (CPU); on the GPU it runs,
and every chain it prints equals the oracle's chain on the same seed, bit for bit."""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "c" / "main_room.c"


def _build(mh, tmp_path, std="c11"):
    exe = tmp_path / f"main_room_{std}"
    subprocess.run(["gcc", f"-std={std}", "-Wall", "-Wextra", "-Werror", "-I", str(ROOT / "include"),
                    str(SRC), "-o", str(exe), str(mh.LIB_PATH),
                    f"-Wl,-rpath,{mh.LIB_PATH.parent}"], check=True)
    return exe


@pytest.mark.parametrize("std", ["c99", "c11"])
def test_harness_compiles_and_links_as_c(mh, tmp_path, std):
    exe = _build(mh, tmp_path, std)
    assert exe.exists()


def _parse(out: str, chains: int, n: int):
    pts = np.zeros((chains, n, 6), dtype=np.float32)
    costs = np.zeros((chains, 8), dtype=np.float32)
    i = -1
    for ln in out.splitlines():
        f = ln.split()
        if ln.startswith("Result "):
            i = int(f[1])
            costs[i] = [float.fromhex(v) for v in f[3:11]]
        elif ln.startswith("Point ["):
            j = int(f[1].strip("[]"))
            pts[i, j] = [float.fromhex(v) for v in f[2:8]]
    assert i == chains - 1
    return pts, costs


@pytest.mark.gpu
@pytest.mark.parametrize("chains", [1, 300])
def test_harness_runs_the_reference_room(mh, orc, hiplib, tmp_path, chains):
    """main()'s call, KernelWrapper(rss, rsa, cfg, clearances, offlimits, vtx, surfaceRectangle,
    &srf, &gpuCfg) with 100 iterations (Kernel.cu:1187-1198), seeded by $MH_SEED, from C."""
    exe = _build(mh, tmp_path)
    seed = 1234567 + chains
    env = dict(os.environ, MH_SEED=str(seed))
    env.pop("MH_DEVICES", None)
    r = subprocess.run([str(exe), str(chains)], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("Target angles are (0.785400,1.963500)")
    pts, costs = _parse(r.stdout, chains, 32)
    ref_pts, ref_costs, _ = orc.run_chains(mh.main_fixture(), chains, 100, seed, threads=8)
    assert np.array_equal(pts.view(np.uint32), ref_pts.view(np.uint32))
    assert np.array_equal(costs.view(np.uint32), ref_costs.view(np.uint32))
