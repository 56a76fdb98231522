import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

import __graft_entry__ as graft  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def mh():
    return graft.load_package()


@pytest.fixture(scope="session")
def orc():
    o = graft.load_oracle()
    o.build()
    return o


@pytest.fixture(scope="session")
def hiplib(mh):
    """libmhgpu.so, built if missing. GPU tests must run the HIP path: no fallback."""
    if not mh.LIB_PATH.exists():
        graft.build()
    return mh.load_library()
