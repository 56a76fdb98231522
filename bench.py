#!/usr/bin/env python3
"""Benchmark: MH chain-steps/s on the 64-object synthetic room (BASELINE.json config 3).

One bench "step" advances every chain of this GPU's shard by --iters MH steps (propose ->
Costs -> accept, Kernel.cu:785-828; 4,000 by default, i.e. four 1,000-step kernel launches),
state resident in HBM/LDS. The driver's `--steps 20 --warmup 5` and the defaults (24 + 1) both
run config 3's full 100,000 MH steps per chain, so mean_final_cost is the config's own.
value = (all ranks' chains) x (timed MH steps) / max-over-ranks wall time.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process
per GPU, chains sharded by global id (chain c always draws Philox subsequence c), no collective
on the data path; after sampling one RCCL all-gather of each rank's 40-byte best-cost summary
selects the global best layout (north_star). Weak scaling: --chains chains per GPU.

Also reported: a VALU roofline for the step kernel (canonical algorithmic
flops F(N,C,R) per chain-step / measured kernel time vs the 157.3 TFLOP/s FP32 vector peak) and
the oracle's restatement of the reference chain timed on this host's cores (cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import __graft_entry__ as graft  # noqa: E402

FP32_VECTOR_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md chip table (== FP32 MFMA peak)
HBM_PEAK_GBS = 8000.0
VALU_LANE_OPS_PEAK = FP32_VECTOR_PEAK_TFLOPS * 1e12 / 2  # lane-operations/s (an FMA is 2 flops)
STEPS_PER_LAUNCH = 1000  # the library's launch chunk (mh_abi.cpp kStepsPerLaunch)


def algorithmic_flops(n: int, c: int, r: int) -> int:
    """canonical flops of one chain-step (full recompute of the accept-relevant
    cost, off-limits excluded; each sqrt/transcendental counts 1)."""
    return 14 * n * n + 10 * c * n + 60 * c + 89 * n + 25 * r + 60


def state_bytes_per_chain(n: int) -> int:
    """HBM bytes one launch moves per chain: pose load + store (6 doubles per object) and the
    64-byte ChainMeta load + store. The room tables are shared and L2-resident."""
    return 2 * (6 * 8 * n) + 2 * 64


def shard(rank: int, chains_per_rank: int):
    """Global chain ids [offset, offset + count) owned by `rank` (weak scaling: every rank owns
    chains_per_rank chains). Chain c always draws Philox subsequence c, so a chain's result does
    not depend on how many ranks there are."""
    return rank * chains_per_rank, chains_per_rank


def summary_record(sum_total: float, best_total: float, best_chain: int, n_chains: int,
                   accepted: int):
    """The per-rank record all-gathered over RCCL (40 bytes of payload as float64)."""
    return [float(sum_total), float(best_total), float(best_chain), float(n_chains),
            float(accepted)]


def combine_records(recs):
    """Combines all-gathered summary records (rows of summary_record) into the job result:
    global best (lowest global chain id on ties), mean final cost, chain and accept counts."""
    best = None
    for r in recs:
        key = (r[1], -r[2])
        if best is None or key > (best[1], -best[2]):
            best = r
    total = sum(int(r[3]) for r in recs)
    return {"best_final_cost": float(best[1]), "best_chain": int(best[2]),
            "mean_final_cost": sum(r[0] for r in recs) / total, "chains": total,
            "accepted": int(sum(r[4] for r in recs))}


def cpu_share():
    """(CPUs this job may use, where that number comes from): the cgroup's CPU quota
    (/sys/fs/cgroup/cpu.max, cgroup v2) when one is set, else $OMP_NUM_THREADS (the GPU pool sets
    it to the one-GPU job's share), else 16."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) / int(period))), f"cgroup cpu.max {quota} {period}"
    except (OSError, ValueError):
        pass
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env), f"OMP_NUM_THREADS={env}"
    return 16, "default (16)"


def host_cores():
    """(threads the CPU baseline uses, nproc, CPUs this process may run on, share source). The
    GPU box grants a one-GPU job a share of a larger machine whose CPUs nproc and the affinity
    mask count in full, so the baseline runs on min(affinity, share) threads (cpu_share) and
    reports every number."""
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = nproc
    share, source = cpu_share()
    return max(1, min(affinity, share)), nproc, affinity, source


def cpu_baseline(room, orc, seed: int, budget_s: float):
    """Oracle chain (the reference's algorithm, Kernel.cu:777-828, OffLimits included as the
    reference computes it every step) on the host's cores, bounded to ~budget_s."""
    threads, nproc, affinity, source = host_cores()
    t0 = time.perf_counter()
    orc.run_chains(room, threads, 20, seed, threads=threads)
    per = (time.perf_counter() - t0) / (threads * 20) * threads  # seconds per chain-step/thread
    steps = max(20, int(budget_s / max(per, 1e-9) / 4))
    chains = 4 * threads
    t0 = time.perf_counter()
    orc.run_chains(room, chains, steps, seed, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": chains * steps / dt, "unit": "chain-steps/s", "cores": threads,
            "kind": "port", "host_nproc": nproc, "host_affinity_cpus": affinity,
            "cpu_share_source": source,
            "sample": f"oracle/mh_oracle.c chain on {room.name}: {chains} chains x {steps} steps"
                      f" ({dt:.1f} s, {threads} threads; nproc {nproc}, {affinity} CPUs in this"
                      f" process's affinity; the job's CPU share from {source})"}


def e2e_wrapper(mh, room, chains: int, iters: int, seed: int):
    """The drop-in entry point end to end (SURVEY.md 8(d) "Also report end-to-end KernelWrapper
    time"): one KernelWrapperSeeded call on host buffers, as the reference's caller makes it
    (Kernel.cu:873-984: room upload, chain setup, `iters` MH steps, the final pass and the copy
    of every chain's points and costs back into the host result), wall-clock timed."""
    import ctypes as C
    lib = mh.load_library()
    g = mh.abi.gpuConfig(chains, 0, 64, 0, 0, iters)
    walls = []
    for k in range(2):  # the process's first call also creates the pooled session (cold)
        t0 = time.perf_counter()
        res = lib.KernelWrapperSeeded(*room.args(), C.byref(g), C.c_uint64(seed + k))
        walls.append(time.perf_counter() - t0)
        if not res:
            raise mh.MHError(mh.last_error(lib))
        lib.KernelFreeResult(res)
    wall = walls[1]
    return {"entry": "KernelWrapperSeeded", "chains": chains, "iterations": iters,
            "wall_s": wall, "chain_steps_per_s": chains * iters / wall,
            "cold_wall_s": walls[0], "cold_chain_steps_per_s": chains * iters / walls[0],
            "result_bytes": chains * (room.n * 24 + 40),
            "note": "host buffers in, host result out (PCIe both ways), a caller's second call "
                    "(the first also sets up the per-device session the library keeps); never "
                    "`value`"}


def library_srchash(mh) -> str | None:
    """The source hash recorded next to the library this process loaded (None for a library
    without one, e.g. an ablate/ variant under $MH_LIB)."""
    lib = Path(os.environ.get("MH_LIB", mh.LIB_PATH))
    stamp = lib.with_name(lib.name + ".srchash")
    return stamp.read_text().strip() if stamp.exists() else None


def pmc_record(n: int, n_chains_per_launch: int, step_kernel: str, srchash: str | None):
    """(record, status): the committed rocprofv3 PMC record of the step kernel
    (profiles/pmc_step_kernel_n<N>.json, written by tools/pmc_summary.py --json) if it was taken
    on this workload AND on a library built from the same sources as the one loaded (its srchash
    stamp), else {} -- a PMC record of another build never describes this one."""
    p = ROOT / "profiles" / f"pmc_step_kernel_n{n}.json"
    if not p.exists():
        return {}, "no PMC record for this room"
    try:
        d = json.loads(p.read_text())
    except Exception as e:  # noqa: BLE001
        return {}, f"unreadable PMC record ({e})"
    k = d.get("kernel", "")
    kind = ("incremental" if "delta" in k else "speculative" if "mh_spec_kernel" in k else
            "full-few" if "mh_kernel<64, 1, 6>" in k else "full")
    if int(d.get("chains_per_launch", -1)) != n_chains_per_launch or kind != step_kernel:
        return {}, "PMC record of another workload"
    if not srchash or d.get("srchash") != srchash:
        return {}, (f"stale: PMC record of library {str(d.get('srchash'))[:12]}, this library "
                    f"{str(srchash)[:12]}")
    return d, f"current (library {srchash[:12]})"


CONFIG_NAMES = {(64, 65536): "config 3: ", (256, 32768): "config 5: ", (8, 1024): "config 2: "}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=24,
                    help="timed bench steps (1 warmup + 24 = the config's 100k MH steps)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--iters", type=int, default=4000, help="MH steps per bench step")
    ap.add_argument("--objects", type=int, default=64)
    ap.add_argument("--chains", type=int, default=65536, help="chains per GPU")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-budget", type=float, default=30.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e-iters", type=int, default=4000,
                    help="MH steps of the end-to-end KernelWrapperSeeded leg (0: skip)")
    ap.add_argument("--collective", action="store_true",
                    help="run the process group and the best-cost all-gather even at world size "
                         "1 (the RCCL leg on device tensors with one GPU; launched without "
                         "torch.distributed.run it rendezvouses on 127.0.0.1)")
    args = ap.parse_args()
    args.iters = max(1, args.iters)
    launches_per_step = -(-args.iters // STEPS_PER_LAUNCH)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    # One process per GPU over RCCL. $MH_BENCH_BACKEND=gloo rehearses the multi-rank path on a
    # box with fewer GPUs than ranks (ranks then share devices round-robin; CPU-side collectives).
    backend = os.environ.get("MH_BENCH_BACKEND", "nccl")
    if backend == "nccl" and world > 1 and torch.cuda.device_count() < world:
        # (one process per GPU: fewer visible GPUs than ranks would fail inside RCCL later)
        raise SystemExit(f"bench.py: {world} ranks over RCCL need {world} GPUs, this process sees "
                         f"{torch.cuda.device_count()} (MH_BENCH_BACKEND=gloo rehearses the "
                         f"multi-rank path on fewer GPUs)")
    device = local_rank if backend == "nccl" else local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    # The collective leg runs whenever there is more than one rank, or on request at one rank.
    use_dist = world > 1 or args.collective
    if use_dist and "MASTER_ADDR" not in os.environ:  # (a plain `python bench.py --collective`)
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0",
                          WORLD_SIZE="1")
    if use_dist:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)
    cdev = f"cuda:{device}" if backend == "nccl" else "cpu"

    mh = graft.load_package()
    mh.load_library()
    room = mh.synthetic_room(args.objects)
    n, c, r = room.n, room.srf.nClearances, room.srf.nRelationships

    # A dedicated (non-null) stream: the kernels and the timing events share it.
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    handle = stream.cuda_stream
    assert handle, "need a non-null HIP stream handle"
    offset, count = shard(rank, args.chains)
    sess = mh.Session(room, count, seed=args.seed, device=device, chain_offset=offset)
    lanes, cpw, step_kernel = sess.step_kernel()
    resident = sess.occupancy()

    for _ in range(args.warmup):
        sess.run(args.iters, handle)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        sess.run(args.iters, handle)
    ev1.record(stream)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1)

    # Final state, summary and the RCCL best-cost all-gather (outside the timed region).
    sess.finalize(handle)
    torch.cuda.synchronize()
    s = sess.summary()
    rec = torch.tensor(summary_record(s.sum_total, s.best_total, s.best_chain, s.n_chains,
                                      s.accepted), dtype=torch.float64,
                       device=cdev)
    times = torch.tensor([wall, kernel_ms], dtype=torch.float64, device=cdev)
    # this rank's identity and timing, so a multi-rank line shows which GPU each rank drove
    props = torch.cuda.get_device_properties(device)
    pci = [getattr(props, k, -1) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id")]
    me = torch.tensor([rank, device, *pci, wall, kernel_ms, offset, count], dtype=torch.float64,
                      device=cdev)
    ranks = None
    if use_dist:
        gathered = [torch.empty_like(rec) for _ in range(world)]
        dist.all_gather(gathered, rec)
        everyone = [torch.empty_like(me) for _ in range(world)]
        dist.all_gather(everyone, me)
        dist.all_reduce(times, op=dist.ReduceOp.MAX)
        recs = torch.stack(gathered).cpu()
        ranks = [dict(zip(("rank", "device", "pci_domain", "pci_bus", "pci_device", "wall_s",
                           "kernel_ms", "chain_offset", "chains"), map(float, e.cpu().tolist())))
                 for e in everyone]
        for d in ranks:
            for k in ("rank", "device", "pci_domain", "pci_bus", "pci_device", "chain_offset",
                      "chains"):
                d[k] = int(d[k])
    else:
        recs = rec.unsqueeze(0).cpu()
    wall, kernel_ms = float(times[0]), float(times[1])
    job = combine_records(recs.tolist())
    total_chains = job["chains"]
    mean_cost, best_cost, best_chain = job["mean_final_cost"], job["best_final_cost"], job["best_chain"]
    accept_rate = job["accepted"] / (total_chains * (args.warmup + args.steps) * args.iters)

    chain_steps = total_chains * args.steps * args.iters
    value = chain_steps / wall
    ms_per_step = wall * 1e3 / args.steps
    launches = args.steps * launches_per_step
    launch_s = kernel_ms / 1e3 / launches  # average duration of one step-kernel launch
    iters_per_launch = args.iters / launches_per_step
    f = algorithmic_flops(n, c, r)
    achieved = args.chains * iters_per_launch * f / launch_s / 1e12
    bytes_launch = args.chains * state_bytes_per_chain(n)

    out = None
    if rank == 0:
        e2e = None
        if world == 1 and args.e2e_iters > 0:
            e2e = e2e_wrapper(mh, room, args.chains, args.e2e_iters, args.seed)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            orc = graft.load_oracle()
            cpu = cpu_baseline(room, orc, args.seed, args.cpu_budget)
        pmc, pmc_status = pmc_record(n, args.chains, step_kernel, library_srchash(mh))
        out = {
            "metric": f"MH chain-steps/sec (whole node) + mean final cost, N={n} objects",
            "value": value,
            "unit": "chain-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64+f32 (reference precision map)",
            "data": "synthetic (SURVEY.md 8(d) room, splitmix64 seed 0x5EED0000+N)",
            "config": {
                "workload": CONFIG_NAMES.get((n, args.chains), "")
                            + f"{n}-object synthetic room, {args.chains} chains per GPU,"
                            f" {args.iters} MH steps per bench step",
                "objects": n, "clearances": c, "relationships": r,
                "chains_per_gpu": args.chains, "global_chains": total_chains,
                "mh_steps_per_step": args.iters,
                "mh_steps_total": (args.warmup + args.steps) * args.iters,
                "lanes_per_chain": lanes, "chains_per_workgroup": cpw,
                "resident_chains_per_cu": resident,
                "step_kernel": step_kernel,
                "parallelism": f"chain-sharded x{world} (RCCL best-cost all-gather)",
            },
            "mean_final_cost": mean_cost,
            "best_final_cost": best_cost,
            "best_chain": best_chain,
            "accepted": job["accepted"],
            "accept_rate": accept_rate,
            "kernel_ms_per_step": kernel_ms / args.steps,
            "kernel_ms_per_launch": launch_s * 1e3,
            "roofline": {
                "bound": "valu",
                "achieved": achieved,
                "peak": FP32_VECTOR_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / FP32_VECTOR_PEAK_TFLOPS,
                "traffic": pmc.get("hbm_bytes_per_launch"),
                "flops_per_chain_step": f,
                "algorithmic_bytes_per_launch": bytes_launch,
                "hbm_frac": bytes_launch / launch_s / 1e9 / HBM_PEAK_GBS,
                # F is the canonical full-recompute count; the executed count is
                # the PMC VALU wavefront instructions per chain-step of this build.
                "executed_valu_wave_insts_per_chain_step": (
                    pmc["valu_wave_insts_per_launch"] / (args.chains * pmc["iters_per_launch"])
                    if pmc.get("valu_wave_insts_per_launch") else None),
                # The executed work against the same peak: VALU lane-operations (wavefront
                # instructions x 64 lanes, from the PMC record) per second of this run's launches,
                # over the 78.6e12 lane-ops/s the 157.3 TFLOP/s FMA peak is made of (256 CUs x
                # 128 lanes x 2.4 GHz). `frac` counts the canonical full-recompute flops F; this
                # counts what the kernel issues (incremental work skips, exact passes add).
                "executed_valu_frac": (
                    pmc["valu_wave_insts_per_launch"] * 64 / launch_s / VALU_LANE_OPS_PEAK
                    if pmc.get("valu_wave_insts_per_launch") else None),
                # VALU issue utilisation of the profiled launch (tools/pmc_summary.py): busy
                # SIMD cycles priced per instruction class / (1024 SIMDs x kernel cycles)
                "valu_issue_util": pmc.get("valu_issue_util"),
                # the tracked record this block reads, and the counter summary it was made from
                "pmc_source": (f"profiles/pmc_step_kernel_n{n}.json" if pmc else None),
                "pmc_profile": pmc.get("profile"),
                "pmc_srchash": pmc.get("srchash"),
                "pmc_status": pmc_status,
            },
            "cpu_baseline": cpu,
            # world > 1: what the collective saw (backend, communicator size) and every rank's
            # device, PCI address and timing; distinct PCI addresses = distinct GPUs
            "distributed": ({
                "backend": dist.get_backend(),
                "world_size": dist.get_world_size(),
                "distinct_gpus": len({(d["pci_domain"], d["pci_bus"], d["pci_device"])
                                      for d in ranks}),
                "ranks": ranks,
            } if use_dist else None),
            "e2e_chain_steps_per_s": e2e["chain_steps_per_s"] if e2e else None,
            "e2e": e2e,
        }
        print(json.dumps(out), flush=True)
    sess.close()
    if use_dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
