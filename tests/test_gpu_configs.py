"""BASELINE.json's configurations at their real lengths, the per-GPU path of the 8-GPU config, and
the reference edges that short runs do not reach -- each chain bit for bit against the oracle
(oracle/mh_oracle.c, the restatement of KernelFolder/Kernel/Kernel.cu:754-828).

* config 1: the console harness's 32-object room through KernelWrapper, 10,000 chains x 100 steps;
* config 2: the 8-object room, all 1,024 chains x 10k steps;
* config 3: 256 chains sampled by global id out of a 65,536-chain, 100k-step session (the
  bench's own session: same room, seed and length), plus the device summary of all 65,536
  chains (the bench's mean_final_cost) against the downloaded costs;
* config 4: one rank's shard (global ids 7*65,536 ...) at 5k steps, every one of the 524,288
  global ids of the 8 shards at 20 steps, the bench.py launcher path (2 gloo ranks, and one
  nccl rank whose RCCL all-gather really executes), and KernelWrapper's in-process $MH_DEVICES
  sharding (unmeasured on 8 GPUs: the driver runs those);
* config 5: 64 chains sampled out of a 32,768-chain, 10k-step session of the 256-object room;
* every chain of configs 3, 4 (all 8 shards) and 5 at 20 steps: the whole population's
  workgroup slots and global id -> Philox subsequence mapping, not a sample;
* the index-n pick (u == 1.0f, Kernel.cu:566-574,598-602) on every RNG path, from a searched
  fixture (tests/golden/find_index_n.py);
* KernelWrapper's $MH_SEED against KernelWrapperSeeded (Kernel.cu:873,943);
* the incremental kernel's list-overflow windows (a room where every Clearance pair overlaps).

Every check asserts zero forked chains and reports the count as a ParityReport warning, which
`pytest -q` keeps in its summary. The long oracle runs leave OffLimits out of the per-step
Costs() (oracle.set_step_offlimits(False)): it never enters totalCosts (Kernel.cu:547), so the
chains and their output costs are the same bit for bit, in about half the time.
"""
import contextlib
import json
import os
import socket
import warnings
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np
import pytest

from parity_util import ParityReport, check_chains, forked_chains

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = json.loads((ROOT / "tests" / "golden" / "golden.json").read_text())
HOST_THREADS = 16  # the GPU box's CPU share per GPU


@contextlib.contextmanager
def _fast_oracle(orc):
    orc.set_step_offlimits(False)
    try:
        yield
    finally:
        orc.set_step_offlimits(True)


def _spread(total, blocks, per):
    """`blocks` block starts of `per` chains spread evenly over [0, total), the last block
    ending at the last chain."""
    return [round(k * (total - per) / (blocks - 1)) for k in range(blocks)]


def _oracle_blocks(orc, room, starts, per, steps, seed, threads_each):
    """Oracle chains [b, b + per) for every b in starts, the blocks run concurrently (ctypes
    releases the GIL); returns (points, costs, global ids) in block order."""
    def one(b):
        return orc.run_chains(room, per, steps, seed, chain_begin=b, threads=threads_each)
    with ThreadPoolExecutor(len(starts)) as ex:
        res = list(ex.map(one, starts))
    ids = np.concatenate([np.arange(b, b + per) for b in starts])
    return (np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res]), ids)


def _session_sampled(mh, orc, room, chains, steps, seed, starts, per, threads_each, offset=0):
    """Runs a full-size session (launches queued asynchronously) while the oracle runs the
    sampled blocks, then returns both."""
    with mh.Session(room, chains, seed=seed, chain_offset=offset) as s, _fast_oracle(orc):
        s.run(steps)
        ref_pts, ref_costs, ids = _oracle_blocks(orc, room, [offset + b for b in starts], per,
                                                 steps, seed, threads_each)
        s.finalize()
        pts, costs = s.download()
        summ = s.summary()
    local = ids - offset
    return pts, costs, summ, pts[local], costs[local], ref_pts, ref_costs, ids


def _in_room(room, pts):
    w = np.float32(room.surface_rectangle[0].x)
    return bool(np.all((pts[..., 0] >= 0) & (pts[..., 0] <= w) & (pts[..., 1] >= 0) &
                       (pts[..., 1] <= w)))


def test_config1_main_fixture_full_size(mh, orc, hiplib, monkeypatch):
    """Config 1: the console harness's room (Kernel.cu:1007-1194, N=32) through
    the reference's own symbol KernelWrapper, 10,000 chains x 100 steps = 1M samples, every
    chain against the oracle ($MH_SEED stands in for time(NULL), Kernel.cu:943)."""
    room = mh.main_fixture()
    chains, steps, seed = 10_000, 100, 20_240_531
    monkeypatch.setenv("MH_SEED", str(seed))
    pts, costs = mh.kernel_wrapper(room, chains, steps)  # seed=None -> KernelWrapper
    ref_pts, ref_costs, _ = orc.run_chains(room, chains, steps, seed, threads=HOST_THREADS)
    check_chains("config 1 (main() room N=32, 10000 x 100, KernelWrapper)", pts, costs,
                 ref_pts, ref_costs, report=True)


def test_config2_full_length(mh, orc, hiplib):
    """Config 2 in full: 8-object room, 1,024 chains x 10,000 steps, every chain."""
    room = mh.synthetic_room(8)
    chains, steps, seed = 1024, 10_000, 42
    pts, costs = mh.kernel_wrapper(room, chains, steps, seed=seed)
    ref_pts, ref_costs, _ = orc.run_chains(room, chains, steps, seed, threads=HOST_THREADS)
    check_chains("config 2 (N=8, 1024 x 10k)", pts, costs, ref_pts, ref_costs, report=True)


def _check_summary(name, summ, costs, offset=0):
    """The device summary (mh_summary_kernel: what bench.py all-gathers and reports as
    mean_final_cost / best_final_cost / best_chain) against the downloaded final costs of every
    chain: the same count, the same best total at the lowest such id, and the mean of all chains'
    totals (a double sum in another order: equal to ~1e-15)."""
    tot = costs[:, 0].astype(np.float64)
    assert summ.n_chains == len(costs)
    assert summ.best_total == costs[:, 0].max()
    assert summ.best_chain == offset + int(np.argmax(costs[:, 0]))
    mean = summ.sum_total / summ.n_chains
    assert mean == pytest.approx(tot.mean(), rel=1e-12, abs=0)
    warnings.warn(f"{name}: device summary of all {len(costs)} chains: mean final total "
                  f"{mean:.9g} (host mean of the downloaded costs {tot.mean():.9g}), best "
                  f"{summ.best_total:.9g} at chain {summ.best_chain}", ParityReport)


def test_config3_full_length_sampled(mh, orc, hiplib):
    """Config 3: a 65,536-chain session run for the config's 100,000 steps -- bench.py's own
    workload (room, seed 42, 25 x 4,000 steps) -- with 256 chains sampled across the id range
    (16 blocks of 16) against the oracle by global id, and the device summary of all chains
    (bench.py's mean_final_cost) against the downloaded costs."""
    room = mh.synthetic_room(64)
    chains, steps, seed = 65536, 100_000, 42
    starts = _spread(chains, 16, 16)
    pts, costs, summ, sp, sc, rp, rc, ids = _session_sampled(
        mh, orc, room, chains, steps, seed, starts, 16, 1)
    assert len(ids) == 256 and len(set(ids.tolist())) == 256
    check_chains("config 3 (N=64, 65536 x 100k, 256 sampled)", sp, sc, rp, rc, ids=ids,
                 report=True)
    _check_summary("config 3", summ, costs)
    assert _in_room(room, pts)


def test_config5_full_length_sampled(mh, orc, hiplib):
    """Config 5: the 256-object room, a 32,768-chain session for 10,000 steps (incremental
    kernel); 64 chains sampled by global id (16 blocks of 4 across the id range) against the
    oracle, and the device summary of all chains against the downloaded costs."""
    room = mh.synthetic_room(256)
    chains, steps, seed = 32768, 10_000, 42
    starts = _spread(chains, 16, 4)
    pts, costs, summ, sp, sc, rp, rc, ids = _session_sampled(
        mh, orc, room, chains, steps, seed, starts, 4, 1)
    assert len(ids) == 64 and len(set(ids.tolist())) == 64
    check_chains("config 5 (N=256, 32768 x 10k, 64 sampled)", sp, sc, rp, rc, ids=ids,
                 report=True)
    _check_summary("config 5", summ, costs)
    assert _in_room(room, pts)


def test_config4_rank7_shard(mh, orc, hiplib):
    """Config 4's per-GPU work on one GPU: rank 7's shard (global ids [7*65536, 8*65536)),
    64 chains sampled against the oracle at the same global ids (unmeasured on 8 GPUs)."""
    room = mh.synthetic_room(64)
    chains, steps, seed, offset = 65536, 5_000, 42, 7 * 65536
    starts = [0, 9360, 18720, 28080, 37440, 46800, 56160, 65528]
    pts, costs, summ, sp, sc, rp, rc, ids = _session_sampled(
        mh, orc, room, chains, steps, seed, starts, 8, 2, offset=offset)
    check_chains("config 4 rank-7 shard (N=64, 65536 x 5k, 64 sampled)", sp, sc, rp, rc,
                 ids=ids, report=True)
    _check_summary("config 4 rank-7 shard", summ, costs, offset=offset)


@pytest.mark.parametrize("name,n,chains,offset", [
    ("config 3", 64, 65536, 0),
    ("config 5", 256, 32768, 0)])
def test_every_chain_short(mh, orc, hiplib, name, n, chains, offset):
    """Every chain of a config's full population, at 20 steps: each workgroup slot, wavefront
    and global id -> Philox subsequence mapping of the launch (one chain per block id,
    Kernel.cu:950) compared bit for bit with the oracle, not a sample. (The long runs above
    compare sampled chains; this covers the whole population at the cost of length.)"""
    room = mh.synthetic_room(n)
    steps, seed = 20, 42
    with mh.Session(room, chains, seed=seed, chain_offset=offset) as s:
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
        summ = s.summary()
    with _fast_oracle(orc):
        ref_pts, ref_costs, ref_acc = orc.run_chains(room, chains, steps, seed,
                                                     chain_begin=offset, threads=HOST_THREADS)
    check_chains(f"{name} (N={n}, all {chains} chains x {steps} steps"
                 + (f", global ids from {offset}" if offset else "") + ")",
                 pts, costs, ref_pts, ref_costs, ids=offset + np.arange(chains), report=True)
    assert summ.accepted == int(np.asarray(ref_acc).sum())
    _check_summary(f"{name} ({steps} steps)", summ, costs, offset=offset)


LONG = pytest.mark.skipif(not os.environ.get("MH_LONG_PARITY"),
                          reason="long parity run (~3 min each): set MH_LONG_PARITY=1")


@LONG
def test_config3_every_chain_1000_steps(mh, orc, hiplib):
    """Every one of config 3's 65,536 chains for a whole 1,000-step launch (the 20-step run above
    is too short to reach the bound's rare paths in proportion: ~1.5% of steps are open and
    ~0.8% recompute the current configuration exactly, so every chain takes them ~20 times
    here), bit for bit against the oracle. Opt-in ($MH_LONG_PARITY=1): ~2.5 min of oracle time on
    16 host threads; its record is committed under profiles/."""
    room = mh.synthetic_room(64)
    chains, steps, seed = 65536, 1000, 42
    with mh.Session(room, chains, seed=seed) as s, _fast_oracle(orc):
        s.run(steps)
        ref_pts, ref_costs, ref_acc = orc.run_chains(room, chains, steps, seed,
                                                     threads=HOST_THREADS)
        s.finalize()
        pts, costs = s.download()
        summ = s.summary()
    check_chains(f"config 3 (N=64, all {chains} chains x {steps} steps)", pts, costs, ref_pts,
                 ref_costs, report=True)
    assert summ.accepted == int(np.asarray(ref_acc).sum())


@LONG
def test_config5_full_length_256_sampled(mh, orc, hiplib):
    """Config 5 at its full 10,000 steps with 256 chains sampled by global id (4x the default
    test's 64), 32 blocks of 8 across the id range. Opt-in ($MH_LONG_PARITY=1)."""
    room = mh.synthetic_room(256)
    chains, steps, seed = 32768, 10_000, 42
    starts = _spread(chains, 32, 8)
    pts, costs, summ, sp, sc, rp, rc, ids = _session_sampled(
        mh, orc, room, chains, steps, seed, starts, 8, 1)
    assert len(set(ids.tolist())) == 256
    check_chains("config 5 (N=256, 32768 x 10k, 256 sampled)", sp, sc, rp, rc, ids=ids,
                 report=True)
    _check_summary("config 5", summ, costs)


def test_config4_every_chain_all_shards(mh, orc, hiplib):
    """Config 4's whole population: all 524,288 global ids, as the 8 ranks of the 8-GPU run
    shard them (rank r: a 65,536-chain session with chain_offset r * 65,536, Kernel.cu:950 one
    block per chain), run one after another on this GPU for 20 steps and compared chain by chain
    with the oracle at the same global ids. Each shard's device summary (what bench.py
    all-gathers) is checked against its downloaded costs, and the combined record
    (bench.combine_records) against the whole population's."""
    sys.path.insert(0, str(ROOT))
    import bench
    room = mh.synthetic_room(64)
    per, ranks, steps, seed = 65536, 8, 20, 42
    forked, compared, recs = 0, 0, []
    dev_sum = ref_sum = 0.0
    best = (-np.inf, -1)
    for r in range(ranks):
        off = r * per
        with mh.Session(room, per, seed=seed, chain_offset=off) as s:
            s.run(steps)  # (queued; the oracle runs meanwhile)
            with _fast_oracle(orc):
                ref_pts, ref_costs, ref_acc = orc.run_chains(room, per, steps, seed,
                                                             chain_begin=off,
                                                             threads=HOST_THREADS)
            s.finalize()
            pts, costs = s.download()
            summ = s.summary()
        bad = forked_chains(pts, costs, ref_pts, ref_costs)
        assert len(bad) == 0, (f"config 4 rank {r}: {len(bad)} of {per} chains forked (global "
                               f"ids {(off + bad[:32]).tolist()})")
        forked += len(bad)
        compared += per
        assert summ.accepted == int(np.asarray(ref_acc).sum())
        _check_summary(f"config 4 rank {r} ({steps} steps)", summ, costs, offset=off)
        recs.append(bench.summary_record(summ.sum_total, summ.best_total, summ.best_chain,
                                         summ.n_chains, summ.accepted))
        dev_sum += float(costs[:, 0].astype(np.float64).sum())
        ref_sum += float(np.asarray(ref_costs)[:, 0].astype(np.float64).sum())
        k = int(np.argmax(costs[:, 0]))
        if costs[k, 0] > best[0]:
            best = (float(costs[k, 0]), off + k)
    job = bench.combine_records(recs)
    assert job["chains"] == compared == ranks * per
    assert (job["best_final_cost"], job["best_chain"]) == best
    mean, ref_mean = dev_sum / compared, ref_sum / compared
    assert job["mean_final_cost"] == pytest.approx(mean, rel=1e-12)
    rel = abs(mean - ref_mean) / abs(ref_mean)
    assert rel <= 1e-4
    warnings.warn(f"config 4 (N=64, all {compared} chains of the 8 shards x {steps} steps, global "
                  f"ids 0..{compared - 1}): {forked} of {compared} chains forked; mean final "
                  f"total {mean:.9g} vs oracle {ref_mean:.9g} (rel {rel:.3g}); combined record "
                  f"best {best[0]:.9g} at chain {best[1]}", ParityReport)


def test_config4_rccl_all_gather_single_gpu(mh, hiplib, tmp_path):
    """The RCCL leg of bench.py executed for real on this box's one GPU: torch.distributed.run
    with one rank, backend nccl, `--collective` lifting the world-size gate, so the communicator
    is created and the summary records are all-gathered as device tensors. The line must name
    the nccl backend, and its record must equal one Session's (unmeasured on 8 GPUs)."""
    n, per, iters, steps, warmup, seed = 16, 4096, 100, 2, 1, 42
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("MH_BENCH_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           str(ROOT / "bench.py"), "--gpus", "1", "--collective", "--objects", str(n),
           "--chains", str(per), "--iters", str(iters), "--steps", str(steps), "--warmup",
           str(warmup), "--seed", str(seed), "--no-cpu-baseline", "--e2e-iters", "0"]
    out = subprocess.run(cmd, env=env, cwd=tmp_path, capture_output=True, text=True, timeout=150)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    rec = json.loads(line)
    d = rec["distributed"]
    assert d["backend"] == "nccl" and d["world_size"] == 1 and d["distinct_gpus"] == 1
    assert [x["rank"] for x in d["ranks"]] == [0]
    room = mh.synthetic_room(n)
    with mh.Session(room, per, seed=seed) as s:
        s.run((steps + warmup) * iters)
        s.finalize()
        summ = s.summary()
    assert rec["best_chain"] == summ.best_chain
    assert rec["best_final_cost"] == float(summ.best_total)
    assert rec["accepted"] == summ.accepted
    assert rec["mean_final_cost"] == pytest.approx(summ.sum_total / per, rel=1e-12)
    warnings.warn(f"RCCL all-gather executed: backend {d['backend']}, world size "
                  f"{d['world_size']}, rank 0 on device {d['ranks'][0]['device']} (PCI bus "
                  f"{d['ranks'][0]['pci_bus']}); record equals one Session's", ParityReport)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_config4_two_rank_bench_equals_one_session(mh, hiplib, tmp_path):
    """bench.py's multi-rank path as the driver launches it (torch.distributed.run, 2 ranks;
    gloo because this box has one GPU): rank -> Session(chain_offset) -> summary -> all-gather
    -> combine_records. The combined record must equal one Session over both shards."""
    n, per, iters, steps, warmup, seed = 16, 2048, 100, 2, 1, 42
    env = dict(os.environ, MH_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           str(ROOT / "bench.py"), "--gpus", "2", "--objects", str(n), "--chains", str(per),
           "--iters", str(iters), "--steps", str(steps), "--warmup", str(warmup),
           "--seed", str(seed), "--no-cpu-baseline"]
    out = subprocess.run(cmd, env=env, cwd=tmp_path, capture_output=True, text=True, timeout=150)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    rec = json.loads(line)
    room = mh.synthetic_room(n)
    with mh.Session(room, 2 * per, seed=seed) as s:
        s.run((steps + warmup) * iters)
        s.finalize()
        _, costs = s.download()
        summ = s.summary()
    assert rec["n_gpus"] == 2 and rec["config"]["global_chains"] == 2 * per
    assert rec["best_chain"] == summ.best_chain
    assert rec["best_final_cost"] == float(summ.best_total)
    assert rec["accepted"] == summ.accepted
    assert rec["mean_final_cost"] == pytest.approx(summ.sum_total / (2 * per), rel=1e-12)
    # the line names what the collective saw: backend, communicator size, each rank's device
    dist_rec = rec["distributed"]
    assert dist_rec["backend"] == "gloo" and dist_rec["world_size"] == 2
    assert [d["rank"] for d in dist_rec["ranks"]] == [0, 1]
    assert [d["chain_offset"] for d in dist_rec["ranks"]] == [0, per]
    assert dist_rec["distinct_gpus"] == 1  # (two ranks share this box's one GPU)


def test_kernelwrapper_mh_devices_sharding(mh, hiplib, monkeypatch):
    """$MH_DEVICES=0,0 (with $MH_DEVICES_ALLOW_DUPLICATES=1: a repeated id is otherwise an error):
    KernelWrapperSeeded shards the call over two host threads and streams (device 0 twice); the
    result must equal the single-device call bit for bit."""
    room = mh.synthetic_room(64)
    chains, steps, seed = 1000, 300, 4711
    monkeypatch.delenv("MH_DEVICES", raising=False)
    p1, c1 = mh.kernel_wrapper(room, chains, steps, seed=seed)
    monkeypatch.setenv("MH_DEVICES", "0,0")
    with pytest.raises(mh.MHError, match="listed twice"):  # (not a multi-GPU run)
        mh.kernel_wrapper(room, 8, 1, seed=seed)
    monkeypatch.setenv("MH_DEVICES", "0,999")
    with pytest.raises(mh.MHError, match="not a device id"):
        mh.kernel_wrapper(room, 8, 1, seed=seed)
    monkeypatch.setenv("MH_DEVICES", "0,0")
    monkeypatch.setenv("MH_DEVICES_ALLOW_DUPLICATES", "1")
    p2, c2 = mh.kernel_wrapper(room, chains, steps, seed=seed)
    assert np.array_equal(p1.view(np.uint32), p2.view(np.uint32))
    assert np.array_equal(c1.view(np.uint32), c2.view(np.uint32))
    monkeypatch.setenv("MH_DEVICES", "0,0,0")  # uneven shards, tracking and tempering groups
    p3, c3 = mh.kernel_wrapper(room, 996, steps, seed=seed, track=2, temps=4, swap_interval=50,
                               beta_min=0.5)
    monkeypatch.delenv("MH_DEVICES")
    p4, c4 = mh.kernel_wrapper(room, 996, steps, seed=seed, track=2, temps=4, swap_interval=50,
                               beta_min=0.5)
    assert np.array_equal(p3.view(np.uint32), p4.view(np.uint32))
    assert np.array_equal(c3.view(np.uint32), c4.view(np.uint32))


def test_kernelwrapper_mh_seed(mh, hiplib, monkeypatch):
    """The reference's own symbol seeds from $MH_SEED (time(NULL) otherwise, Kernel.cu:943):
    KernelWrapper with MH_SEED=s equals KernelWrapperSeeded(s)."""
    room = mh.main_fixture()
    monkeypatch.setenv("MH_SEED", "123456789")
    p1, c1 = mh.kernel_wrapper(room, 256, 200)  # seed=None -> KernelWrapper
    p2, c2 = mh.kernel_wrapper(room, 256, 200, seed=123456789)
    assert np.array_equal(p1.view(np.uint32), p2.view(np.uint32))
    assert np.array_equal(c1.view(np.uint32), c2.view(np.uint32))


STEP_PATHS = [  # (name, env): every RNG path a chain can take (speculative: N <= 8 only)
    ("full L=64 WaveRng", {"MH_DELTA": "0", "MH_SPEC": "0"}),
    ("full L=32 ChainRng", {"MH_DELTA": "0", "MH_LANES": "32", "MH_SPEC": "0"}),
    ("incremental WaveRng", {"MH_DELTA": "1", "MH_SPEC": "0"}),
    ("incremental WaveRng 1-chain workgroups", {"MH_DELTA": "1", "MH_DELTA_WAVES": "1",
                                                "MH_SPEC": "0"}),
    ("speculative", {"MH_SPEC": "1"}),
]


# The index-n pick needs nObjs >= 33 (tests/test_oracle.py test_index_n_needs_33_objects), and
# the speculative kernel serves rooms of at most 8 objects, so it never meets one.
INDEX_N_PATHS = [p for p in STEP_PATHS if p[0] != "speculative"]


@pytest.mark.parametrize("path", INDEX_N_PATHS, ids=[p[0] for p in INDEX_N_PATHS])
@pytest.mark.parametrize("case", GOLDEN["index_n"], ids=lambda c: f"chain{c['chain']}")
def test_index_n_pick_redrawn(mh, orc, hiplib, monkeypatch, case, path):
    """A chain whose pick draws u == 1.0f: generateRandomIntInRange(63, 0) gives 64 = nObjs
    (Kernel.cu:566-574), redrawn like a frozen object. The oracle must see the event; the device
    must reproduce the chain bit for bit on every step kernel and RNG path that serves N >= 33."""
    for k, v in path[1].items():
        monkeypatch.setenv(k, v)
    room = mh.synthetic_room(case["n"])
    cid, steps, seed = case["chain"], case["steps"], case["seed"]
    orc.index_n_draws(reset=True)
    rp, rc, _ = orc.run_chains(room, 1, steps, seed, chain_begin=cid)
    assert orc.index_n_draws() >= 1
    with mh.Session(room, 1, seed=seed, chain_offset=cid) as s:
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
    check_chains(f"index-n chain {cid} ({path[0]})", pts, costs, rp, rc, ids=[cid])


# (the speculative kernel serves rooms of at most 8 objects: only the N = 8 fixture reaches it)
U1_CASES = [(c, p) for c in GOLDEN["u1_accept"] for p in STEP_PATHS
            if p[0] != "speculative" or c["n"] <= 8]


@pytest.mark.parametrize("case,path", U1_CASES,
                         ids=[f"N{c['n']}-chain{c['chain']}-{p[0]}" for c, p in U1_CASES])
def test_accept_draw_one_rejects_uphill(mh, orc, hiplib, monkeypatch, case, path):
    """A chain whose Accept draws u == 1.0f (the (0, 1] uniform's top value) against an uphill
    proposal: the threshold min(1, exp(...)) is exactly 1, so Accept rejects (Kernel.cu:706-713).
    The rejection bound must not certainly accept it (round 2's bound did; found by
    tools/bound_check.py). Fixture from tests/golden/find_u1_accept.py; bit for bit against the
    oracle on every step kernel and RNG path."""
    for k, v in path[1].items():
        monkeypatch.setenv(k, v)
    room = mh.synthetic_room(case["n"])
    cid, steps, seed = case["chain"], case["steps"], case["seed"]
    orc.u1_uphill_draws(reset=True)
    rp, rc, _ = orc.run_chains(room, 1, steps, seed, chain_begin=cid)
    assert orc.u1_uphill_draws() >= 1
    with mh.Session(room, 1, seed=seed, chain_offset=cid) as s:
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
    check_chains(f"u == 1.0f uphill chain {cid} N={case['n']} ({path[0]})", pts, costs, rp, rc,
                 ids=[cid])


def _crowded_room(mh, n):
    """Every clearance box overlaps every object box at every reachable pose: a 0.5 m room
    (translations clamp to it, Kernel.cu:613-630) and boxes of 0.5-2 m."""
    room = mh.synthetic_room(n)
    w = 0.5
    for k, (x, y) in enumerate([(w, w), (w, 0.0), (0.0, 0.0), (0.0, w)]):
        room.surface_rectangle[k].x, room.surface_rectangle[k].y = x, y
    rng = np.random.default_rng(n)
    for i in range(n):
        room.cfg[i].x, room.cfg[i].y = rng.uniform(0, w, size=2)
    room.srf.centroidX = room.srf.centroidY = w
    room.srf.focalX, room.srf.focalY = w / 2, w
    return room


@pytest.mark.parametrize("waves", ["", "3"])
def test_incremental_list_overflow_windows(mh, orc, hiplib, monkeypatch, waves):
    """The incremental kernel sums Clearance / SurfaceArea lists longer than its LDS capacity
    (4*NP and NP terms, mh_device.h make_delta_layout) in windows rebuilt in place. Here all
    C*N Clearance pairs are non-zero at every step (C*N = 6,400 >> 4*NP = 768), so every
    step takes that path; bit for bit against the oracle (the default workgroup and a 3-chain
    one, so chains of a workgroup run at different speeds)."""
    monkeypatch.setenv("MH_DELTA", "1")
    if waves:
        monkeypatch.setenv("MH_DELTA_WAVES", waves)
    n = 160
    room = _crowded_room(mh, n)
    c = room.srf.nClearances
    np_pad = (n + 63) // 64 * 64
    assert c * n > 4 * np_pad  # the list cannot fit: windows on every step
    chains, steps, seed = 16, 120, 160
    with mh.Session(room, chains, seed=seed) as s:
        assert s.step_kernel()[2].split("-")[0] == "incremental" and s.step_kernel()[0] == 64
        if waves:
            assert s.step_kernel()[1] == int(waves)
        s.run(steps)
        s.finalize()
        pts, costs = s.download()
    rp, rc, _ = orc.run_chains(room, chains, steps, seed, threads=HOST_THREADS)
    # the final states still have (nearly) every pair non-zero, far past the capacity
    assert min(_nonzero_clearance_pairs(room, rp[k]) for k in range(chains)) > 4 * np_pad
    check_chains(f"crowded N={n} incremental waves={waves or 'default'}", pts, costs, rp, rc)


def _nonzero_clearance_pairs(room, pts):
    """Non-zero ClearanceCosts pairs (Kernel.cu:408-431) of one configuration (float points),
    with minValue's untranslated first x (:371)."""
    v = np.array([(q.x, q.y) for q in room.vertices])

    def box(p1, tx, ty):
        q = v[p1:p1 + 4]
        return (min(q[0, 0], *(q[1:, 0] + tx)), (q[:, 1] + ty).min(), (q[:, 0] + tx).max(),
                (q[:, 1] + ty).max())
    objs = [box(room.offlimits[j].point1Index, pts[j, 0], pts[j, 1]) for j in range(room.n)]
    cnt = 0
    for i in range(room.srf.nClearances):
        s = room.clearances[i].SourceIndex
        a = box(room.clearances[i].point1Index, pts[s, 0], pts[s, 1])
        for b in objs:
            cnt += max(a[0], b[0]) < min(a[2], b[2]) and max(a[1], b[1]) < min(a[3], b[3])
    return cnt


def test_kernelwrapper_pooled_sessions(mh, orc, hiplib):
    """KernelWrapper reuses its per-device sessions across calls (mh_abi.cpp "session cache"):
    the stream, buffers and geometry of one call serve the next. A sequence that grows and
    shrinks the room, the chain count and the options -- each call checked bit for bit against
    the oracle -- shows no state leaks from one call into the next."""
    calls = [  # (objects, chains, steps, seed, kwargs)
        (8, 256, 300, 11, {}),
        (64, 96, 120, 12, {}),                       # larger room, fewer chains
        (8, 1024, 200, 13, {}),                      # more chains than any buffer so far
        (8, 256, 300, 11, {}),                       # the first call again: same result
        (16, 128, 150, 14, {"track": mh.abi.MH_TRACK_LOWEST}),
        (16, 128, 150, 15, {"rng": mh.abi.MH_RNG_CURAND_XORWOW}),
        (12, 120, 160, 16, {"temps": 4, "swap_interval": 10, "beta_min": 0.5}),
        (5, 64, 0, 17, {}),                          # zero steps: the input poses
    ]
    first = None
    for n, chains, steps, seed, kw in calls:
        room = mh.synthetic_room(n)
        pts, costs = mh.kernel_wrapper(room, chains, steps, seed=seed, **kw)
        okw = {k: v for k, v in kw.items()}
        if "rng" in okw:
            okw["rng"] = 1
        rp, rc, _ = orc.run_chains(room, chains, steps, seed, threads=HOST_THREADS, **okw)
        check_chains(f"pooled KernelWrapper N={n} {chains}x{steps} {kw}", pts, costs, rp, rc)
        if first is None:
            first = (pts, costs)
        elif (n, chains, steps, seed, kw) == calls[0]:
            assert np.array_equal(pts.view(np.uint32), first[0].view(np.uint32))


def test_kernelwrapper_pool_follows_overrides(mh, orc, hiplib, monkeypatch):
    """A pooled session keeps its kernel choice only while the tuning overrides are unchanged
    (ADVICE round 5): two calls of the same room shape and chain count, one under $MH_SPEC=1 and
    one under $MH_SPEC=0, must run different step kernels (and give the same chains); likewise
    $MH_LANES. KernelReleaseCache() then frees the idle sessions, and the next call builds a new
    one with the same result."""
    room = mh.synthetic_room(8)
    chains, steps, seed = 512, 200, 77
    rp, rc, _ = orc.run_chains(room, chains, steps, seed, threads=HOST_THREADS)
    got = {}
    for spec in ("1", "0"):
        monkeypatch.setenv("MH_SPEC", spec)
        pts, costs = mh.kernel_wrapper(room, chains, steps, seed=seed)
        got[spec] = mh.wrapper_step_kernel()
        check_chains(f"pooled KernelWrapper MH_SPEC={spec}", pts, costs, rp, rc)
    assert got["1"][1] == "speculative" and got["0"][1] != "speculative"
    monkeypatch.setenv("MH_SPEC", "0")
    room64 = mh.synthetic_room(64)
    rp, rc, _ = orc.run_chains(room64, 64, 50, seed, threads=HOST_THREADS)
    lanes = []
    for want in ("64", "32"):
        monkeypatch.setenv("MH_LANES", want)
        monkeypatch.setenv("MH_DELTA", "0")
        pts, costs = mh.kernel_wrapper(room64, 64, 50, seed=seed)
        lanes.append(mh.wrapper_step_kernel()[0])
        check_chains(f"pooled KernelWrapper MH_LANES={want}", pts, costs, rp, rc)
    assert lanes == [64, 32]
    assert mh.release_cache() >= 1
    assert mh.release_cache() == 0
    pts, costs = mh.kernel_wrapper(room64, 64, 50, seed=seed)
    check_chains("KernelWrapper after KernelReleaseCache", pts, costs, rp, rc)
