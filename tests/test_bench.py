"""bench.py's host logic without a GPU: the PMC record is used only for the library it profiled
(its source-hash stamp), and a multi-rank RCCL run with fewer GPUs than ranks fails loudly."""
import json
import os
import subprocess
import sys
from pathlib import Path

import bench

ROOT = Path(__file__).resolve().parents[1]


def _record(tmp_path, monkeypatch, **fields):
    prof = tmp_path / "profiles"
    prof.mkdir(exist_ok=True)
    rec = {"kernel": "void mh::mh_kernel<64, 1, 1>(mh::LaunchArgs)", "chains_per_launch": 65536,
           "hbm_bytes_per_launch": 1.0, "srchash": "abc123"}
    rec.update(fields)
    (prof / "pmc_step_kernel_n64.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "ROOT", tmp_path)


def test_pmc_record_current_only_for_its_library(tmp_path, monkeypatch):
    _record(tmp_path, monkeypatch)
    d, status = bench.pmc_record(64, 65536, "full", "abc123")
    assert d["hbm_bytes_per_launch"] == 1.0 and status.startswith("current")
    d, status = bench.pmc_record(64, 65536, "full", "def456")
    assert d == {} and status.startswith("stale")
    d, status = bench.pmc_record(64, 65536, "full", None)
    assert d == {} and status.startswith("stale")


def test_pmc_record_without_stamp_is_stale(tmp_path, monkeypatch):
    _record(tmp_path, monkeypatch, srchash=None)
    d, status = bench.pmc_record(64, 65536, "full", "abc123")
    assert d == {} and "stale" in status


def test_pmc_record_of_another_workload(tmp_path, monkeypatch):
    _record(tmp_path, monkeypatch)
    assert bench.pmc_record(64, 1024, "full", "abc123")[0] == {}
    assert bench.pmc_record(64, 65536, "incremental", "abc123")[0] == {}
    assert bench.pmc_record(256, 65536, "full", "abc123")[1] == "no PMC record for this room"


def test_nccl_with_too_few_gpus_fails_loudly():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT="29555", MH_BENCH_BACKEND="nccl")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "need 2 GPUs" in r.stderr


def test_committed_pmc_records_are_stamped():
    """Every committed PMC record carries the source hash of the library it profiled."""
    for p in (ROOT / "profiles").glob("pmc_step_kernel_n*.json"):
        d = json.loads(p.read_text())
        assert d.get("srchash"), p.name
