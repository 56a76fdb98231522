"""The rejection bound's decisions verified directly: the self-checking build
libmhgpu_check.so (-DMH_CHECK=1, built by __graft_entry__.build()) runs real chains and, for
every proposal the bound decides, also computes the exact costs and checks that the exact total
lies in the bound's interval, that the current total lies in the interval carried after a
certain acceptance, and that every certain REJECT / ACCEPT is Accept's own decision
(Kernel.cu:706-713). Rooms: configs 2, 3 and 5, wrapped angle ranges, more relationships than
objects, negated weights and poses far outside the proven symmetry range; both step kernels.
Run in a child process (tools/bound_check.py --quick), so the product library is not loaded
beside it."""
import re
import subprocess
import sys
import warnings
from pathlib import Path

import pytest

from parity_util import ParityReport

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def test_bound_decisions_verified_against_exact_costs(mh):
    lib = mh.LIB_PATH.with_name("libmhgpu_check.so")
    assert lib.exists(), "run __graft_entry__.build() (it builds libmhgpu_check.so)"
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "bound_check.py"), "--quick"],
                         capture_output=True, text=True, timeout=280, cwd=ROOT)
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("[bound]")]
    checked = sum(int(m.group(1)) for ln in lines
                  for m in [re.search(r"(\d+) bound decisions checked", ln)] if m)
    warnings.warn(f"bound check: {checked} decisions verified over {len(lines)} runs; "
                  + "; ".join(ln[8:] for ln in lines if "violations 0" not in ln), ParityReport)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    assert len(lines) >= 12 and checked > 1_000_000
    assert all("violations 0" in ln for ln in lines), "\n".join(lines)
