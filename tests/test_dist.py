"""The multi-GPU path of bench.py without GPUs: world_size 2 over gloo. Each rank runs its shard
of chains (here with the oracle, standing in for the device session) and the per-rank summary
records are all-gathered and combined exactly as bench.py does over RCCL. The job result must
equal a single-process run of all chains (chain c draws subsequence c on any rank)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench

CHAINS_PER_RANK, STEPS, SEED, N = 6, 40, 123, 12


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _summary(costs, acc, offset):
    tot = costs[:, 0]
    best = int(np.argmax(tot))  # first max = lowest id
    return bench.summary_record(tot.astype(np.float64).sum(), tot[best], offset + best,
                                len(tot), int(acc.sum()))


def _worker(rank, world, port, out_q):
    import __graft_entry__ as graft
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mh, orc = graft.load_package(), graft.load_oracle()
    room = mh.synthetic_room(N)
    offset, count = bench.shard(rank, CHAINS_PER_RANK)
    _, costs, acc = orc.run_chains(room, count, STEPS, SEED, chain_begin=offset)
    rec = torch.tensor(_summary(costs, acc, offset), dtype=torch.float64)
    gathered = [torch.empty_like(rec) for _ in range(world)]
    dist.all_gather(gathered, rec)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        out_q.put((bench.combine_records(torch.stack(gathered).tolist()), float(t)))
    dist.destroy_process_group()


def test_two_rank_gloo_matches_single_process(mh, orc):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.start_processes(_worker, args=(world, _free_port(), q), nprocs=world, join=True,
                       start_method="spawn")
    job, tmax = q.get()
    assert tmax == world
    room = mh.synthetic_room(N)
    _, costs, acc = orc.run_chains(room, world * CHAINS_PER_RANK, STEPS, SEED)
    ref = bench.combine_records([_summary(costs, acc, 0)])
    assert job["chains"] == ref["chains"] == world * CHAINS_PER_RANK
    assert job["best_chain"] == ref["best_chain"]
    assert job["best_final_cost"] == ref["best_final_cost"]
    assert job["accepted"] == ref["accepted"]
    assert job["mean_final_cost"] == pytest.approx(ref["mean_final_cost"], rel=1e-12)


def test_combine_tie_breaks_on_lowest_chain():
    recs = [bench.summary_record(10.0, 5.0, 7, 4, 3), bench.summary_record(12.0, 5.0, 2, 4, 1)]
    job = bench.combine_records(recs)
    assert job["best_chain"] == 2 and job["chains"] == 8 and job["accepted"] == 4
    assert job["mean_final_cost"] == 22.0 / 8


def test_shards_tile_the_chain_range():
    ids = [c for r in range(4) for c in range(*(lambda o, n: (o, o + n))(*bench.shard(r, 5)))]
    assert ids == list(range(20))
