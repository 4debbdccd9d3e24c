"""Headline benchmark: commit-index updates/sec for 1M Raft groups x 3 replicas
(BASELINE.json configs[3]'s shape), one device pass per step, inputs resident in HBM.

A step = one pass of the batched raft step over every replica of every group:
leaders ingest the previous pass's ReplicateResp batch, run the quorum commit
and propose one 16-byte entry; followers log-match the previous pass's
Replicate batch. Messages go device-to-device through mailbox spaces (no host
round trip). In steady state every group's leader advances committed by one
index per pass; `value` counts those advances (device stats) per second.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process
per GPU, each owning its own 1M groups sharded by clusterID ("scaling": "weak",
no data-path collective: the groups are independent, partition.go:34-36).
--placement spread is BASELINE config 4's synthetic multi-replica variant:
replica r of a group homed on rank h lives on rank (h + r) % N and the
Replicate/ReplicateResp mailboxes cross GPUs with one RCCL all_to_all_single
per pass (dragonboat_amd/exchange.py).

Roofline accounting: algorithmic bytes are SURVEY.md §8d's
per-unit figures times the units the launch processed, counted on the device:
69 B per message a leader ingests (B_resp), 65 B per message a leader emits
(B_emit), 122 + 16 n B per Replicate of n entries a follower matches
(B_match with ov + ap = n), and 8R + 48 B per group for the quorum commit
(B_commit). In steady state each follower gets two Replicates per pass (the
commit-carrying broadcast of raft.go:1214 and the proposal's), so one
group-round is 1,128 B at R = 3; SURVEY's B_round (616 B) assumes one, and is
reported beside it as "canonical_round_bytes".
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# SURVEY.md §8d canonical algorithmic bytes of one group-round (reference field
# widths): B_round(R) = (R-1)*(69 + 65 + 138) + 8R + 48 -> R=3: 616 B.
def b_round(R):
    return (R - 1) * (69 + 65 + 138) + 8 * R + 48


B_RESP, B_EMIT, B_MATCH0, B_ENTRY = 69, 65, 122, 16


def algorithmic_bytes(st, groups, R, passes):
    """SURVEY.md §8d per-unit bytes x the units counted by the device stats over `passes` passes."""
    follower_in = st["msgs_in"] - st["leader_msgs_in"]
    return (B_RESP * st["leader_msgs_in"] + B_EMIT * st["leader_msgs_out"] + B_MATCH0 * follower_in
            + B_ENTRY * st["replicate_entries"] + (8 * R + 48) * groups * passes)


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, spec


def stream_copy_gbs(torch, dev, nbytes=1 << 30, reps=5):
    """Achievable HBM bandwidth on this box: a device-to-device copy of 1 GiB
    (read + write = 2 GiB moved per copy, past the 256 MiB Infinity Cache),
    best of `reps`, HIP events. Reported beside the spec peak, never instead of it."""
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    a.fill_(1)
    b.copy_(a)
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    del a, b
    return 2 * nbytes / (best * 1e-3) / 1e9


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--groups", type=int, default=1_000_000, help="groups per GPU")
    ap.add_argument("--replicas", type=int, default=3)
    ap.add_argument("--placement", choices=["local", "spread"], default=None)
    ap.add_argument("--cpu-baseline", choices=["on", "off"], default="on")
    ap.add_argument("--cpu-groups", type=int, default=20000)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--check", action="store_true", help="verify the final state against a host replay")
    return ap.parse_args()


def cpu_baseline(args, R):
    """The oracle (C++ restatement of the reference Go step, faithful data
    structures) on a bounded sample of the same workload, host cores only."""
    import numpy as np
    from dragonboat_amd import abi, populations as P
    from oracle.pyoracle import OraclePopulation
    G = args.cpu_groups
    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    peers = P.make_groups(G, R, seed=2)
    topo = P.Topology(G, R)
    pop = OraclePopulation(peers, R)
    msgs = np.zeros(0, abi.MESSAGE)
    # warm to steady state (2 passes), then time
    for k in range(2):
        loc = P.propose_locals(R * G, np.arange(G), pass_index=k)
        o = pop.step(msgs, loc, threads=threads)
        msgs = topo.route_messages(o["msgs"])
    passes, t_step, commits = 0, 0.0, 0
    before = pop.export()["committed"][:G].copy()
    t_end = time.time() + 10.0
    k = 2
    while time.time() < t_end or passes < 2:
        loc = P.propose_locals(R * G, np.arange(G), pass_index=k)
        t0 = time.perf_counter()
        o = pop.step(msgs, loc, threads=threads)
        t_step += time.perf_counter() - t0
        msgs = topo.route_messages(o["msgs"])
        pop.commit_all()
        passes += 1
        k += 1
    after = pop.export()["committed"][:G]
    commits = int(np.sum(after - before))
    return {"value": commits / t_step, "unit": "commit-index updates/s", "cores": threads,
            "kind": "port",
            "sample": f"{G} groups x {R} replicas, {passes} passes, oracle raft step timed "
                      f"(message routing and persistence excluded), {threads} threads"}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs (not used by the driver): GR_BENCH_BACKEND=gloo with
    # GR_BENCH_ONE_DEVICE=1 runs N ranks on one GPU to exercise the N > 1 path
    # of this script on a one-GPU box (RCCL itself refuses two ranks per device).
    backend = os.environ.get("GR_BENCH_BACKEND", "nccl")
    ordinal = 0 if os.environ.get("GR_BENCH_ONE_DEVICE") == "1" else local_rank
    torch.cuda.set_device(ordinal)  # before the process group: RCCL binds the current device
    dev = torch.device("cuda", ordinal)
    cdev = dev if backend == "nccl" else torch.device("cpu")  # where the control collectives run
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from dragonboat_amd import abi, populations as P
    from dragonboat_amd.engine import Engine
    from dragonboat_amd.exchange import build_exchange

    R = args.replicas
    S = R
    G = args.groups
    placement = args.placement or "local"
    ex = build_exchange(G, R, S, world, rank, placement)
    n = ex.n_peers
    eng = Engine(n, S, device=ordinal)
    eng.load(ex.peers)
    eng.bind_routes(ex.in_pos, ex.out_pos)
    loc = P.propose_locals(n, ex.leader_slots, pass_index=0)
    eng.set_locals(loc)
    spaces = ex.allocate(eng, dev)
    stream = torch.cuda.current_stream()

    def one_pass(k):
        ex.step(eng, spaces, k, stream)

    for k in range(args.warmup):
        one_pass(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    eng.reset_stats()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ex.step(eng, spaces, args.warmup + k, stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    st = eng.stats()
    # Per-kernel durations for the roofline: the same passes once more, outside the
    # timed region, with HIP events around each kernel (recorded inside the library
    # on `stream`), so the events add nothing to `value`.
    eng.timing_begin()
    for k in range(args.steps):
        ex.step(eng, spaces, args.warmup + args.steps + k, stream)
    tm = eng.timing_end()
    copy_gbs = stream_copy_gbs(torch, dev)
    commits = st["leader_commits"]
    esc = st["escalations"]
    if world > 1:
        t = torch.tensor([commits, esc], dtype=torch.float64, device=cdev)
        dist.all_reduce(t)
        commits, esc = int(t[0].item()), int(t[1].item())
    value = commits / elapsed
    passes = max(1, tm["passes"])
    kavg = tm["fast_ms"] / passes  # the dominant kernel
    gavg = tm["general_ms"] / passes
    groups_total = G * world
    alg = algorithmic_bytes(st, G, R, args.steps) / args.steps  # per launch (this rank)
    achieved = alg / (kavg * 1e-3) / 1e9  # GB/s: algorithmic bytes of the launch / its time
    canon = b_round(R) * G
    if rank == 0:
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_latest.json")
        if os.path.exists(pmc):  # tools/profile.sh: calibrated FETCH_SIZE + WRITE_SIZE of this kernel
            try:
                from dragonboat_amd.build import source_digest
                rec = json.load(open(pmc))
                if rec.get("groups") == G and rec.get("replicas") == R and \
                        rec.get("source_digest") == source_digest():  # measured on this very kernel
                    traffic = rec.get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        line = {
            "metric": "commit-index updates/sec (1M groups x 3 replicas) + achieved HBM GB/s",
            "value": value,
            "unit": "commit-index updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic steady-state groups (BASELINE config 4 shape), 16-B proposals",
            "config": {"workload": f"{G} groups x {R} replicas per GPU, replicas {placement}, "
                                   f"1 proposal per leader per pass", "groups_total": groups_total,
                       "replicas": R, "placement": placement},
            "escalations": esc,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": f"gr_fast_kernel<{S}>", "kernel_ms": kavg,
                         "algorithmic_bytes_per_launch": alg,
                         "units_per_launch": {k: st[k] / args.steps for k in
                                              ("leader_msgs_in", "leader_msgs_out", "msgs_in",
                                               "replicate_entries")},
                         "canonical_round_bytes": canon,
                         "canonical_frac": canon / (kavg * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "hbm_traffic_GBs": (traffic / (kavg * 1e-3) / 1e9) if traffic else None,
                         "stream_copy_GBs": copy_gbs,
                         "hbm_traffic_frac_of_stream_copy": ((traffic / (kavg * 1e-3) / 1e9) / copy_gbs)
                         if traffic else None,
                         "general_kernel_ms": gavg,
                         "bailed_lanes_per_pass": tm["bailed_lanes"] / passes},
        }
        if args.cpu_baseline == "on" and world == 1:
            try:
                line["cpu_baseline"] = cpu_baseline(args, R)
            except Exception as e:  # baseline is reported, not required
                line["cpu_baseline"] = {"value": None, "error": str(e)}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
