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

Roofline accounting: `achieved` = the algorithmic bytes one
launch must move at this engine's encoding, over the lean kernels' HIP-event
duration. The unit is one group-round; its bytes are counted field by field
from the steady lanes' loads and stores (gr_steady.h; 300 B at R = 3: leader
62 B loaded + 52 B stored, each follower 54 + 39 B), and a launch processes one
group-round per leader commit. PMC checks it (`traffic`).
SURVEY.md §8d's canonical count at reference field widths, B_round(R) =
(R-1)(69+65+138) + 8R + 48 = 616 B at R = 3, is reported beside it as
`canonical_achieved`/`canonical_frac`: it counts bytes the kernels never move,
so at this pass time it implies more than the HBM can physically deliver and
is not a roofline position. `traffic` is the calibrated FETCH_SIZE +
WRITE_SIZE of the same kernels (profiles/pmc_latest.json, used only when its
source digest matches this build) and `traffic_frac` the physical rate over
the 8 TB/s peak. The reference-width per-message count (two Replicates and two
acks per follower per round, 1,128 B/group) is reported as
`reference_width_bytes_per_launch` only. `copy_f4_GBs` is tools/hbm_calib's
float4 copy on the same box (achievable HBM).

Beside the headline (rank 0, N = 1): `host_path` times gr_step with host records
(the C-ABI call a Go step worker makes, PCIe-inclusive), and `cpu_baseline`
follows BASELINE.md's CPU protocol on bounded samples.
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

# Bytes one steady group-round moves at this engine's encoding (gr_steady.h,
# loopback routes, R = 3), load by load and store by store. The
# two messages of each steady mailbox travel shared (gr_layout.h MB_SHARED:
# message 0's hot fields only):
#   leader   loads  hdr, term, committed, lastIndex 32 + locals word 4
#                   + 2 ack mailboxes x (count 1 + term word 4 + LogIndex 8)
#                   (match rows: header bits H_MP, gr_layout.h)          =  62
#            stores committed 8 + lastIndex 8
#                   + 2 out mailboxes x (LogIndex 8 + Commit offset 4
#                   + term word 4 + count 1) + proposal result 1 + flags 1 =  52
#   follower loads  core 32 + locals word 4 + 2 count bytes + term word 4
#                   + LogIndex 8 + Commit offset 4                       =  54
#            stores committed 8 + lastIndex 8 + ack mailbox (LogIndex 8
#                   + term word 4 + count 1) + other count 1
#                   + append_from 8 + flags 1                            =  39
# = 62 + 52 + 2 x (54 + 39) = 300 B per group-round.
ENCODED_ROUND_BYTES = {3: 300}


def reference_width_bytes(st, groups, R, passes):
    """SURVEY.md §8d per-message bytes x the messages counted by the device over `passes`
    passes (two Replicates and two acks per follower per round: 1,128 B/group at R = 3)."""
    follower_in = st["msgs_in"] - st["leader_msgs_in"]
    return (B_RESP * st["leader_msgs_in"] + B_EMIT * st["leader_msgs_out"] + B_MATCH0 * follower_in
            + B_ENTRY * st["replicate_entries"] + (8 * R + 48) * groups * passes)


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--launch", choices=["stream", "graph"], default="stream",
                    help="timed passes launched kernel by kernel, or replayed from the library's two-pass HIP "
                         "graph (gr_graph_capture / gr_graph_replay; local placement, even --steps)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--groups", type=int, default=1_000_000, help="groups per GPU")
    ap.add_argument("--replicas", type=int, default=3)
    ap.add_argument("--placement", choices=["local", "spread"], default=None,
                    help="default: local at N=1, spread (BASELINE config 4) at N>1")
    ap.add_argument("--banks", type=int, default=None,
                    help="engines per rank whose exchanges overlap each other's passes (spread default 2)")
    ap.add_argument("--cpu-baseline", choices=["on", "off"], default="on")
    ap.add_argument("--cpu-groups", type=int, default=20000)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="T of the CPU baseline (0: nproc capped by affinity and the cgroup quota)")
    ap.add_argument("--cpu-seconds", type=float, default=40.0, help="CPU baseline time budget (all legs)")
    ap.add_argument("--host-path", choices=["on", "off"], default="on",
                    help="also time gr_step with host records (N=1, rank 0)")
    ap.add_argument("--host-passes", type=int, default=4)
    ap.add_argument("--host-partitions", type=int, default=2,
                    help="concurrent step workers (engines) of the compact host-path leg")
    ap.add_argument("--host-pipeline-partitions", type=int, default=4,
                    help="partitions of the pipelined compact host-path leg (begin/end halves)")
    ap.add_argument("--check", action="store_true", help="verify the final state against a host replay")
    return ap.parse_args()


def cpu_info():
    """Host CPU description for the baseline (nproc + lscpu model)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "lscpu_model": model}


def _oracle_rate(peers, topo, R, locals_fn, threads, seconds, inject=None, drop=None):
    """Oracle raft step (C++ restatement of internal/raft, faithful data structures)
    over a population for about `seconds`: returns (leader commits/s, groups
    stepped/s, passes). Message routing, persistence and injection are untimed."""
    import numpy as np
    from dragonboat_amd import abi
    from oracle.pyoracle import OraclePopulation
    pop = OraclePopulation(peers, R)
    pop.set_truncate_runs()  # long churn runs build >2-run Replicates; the records carry a prefix
    pop.rehome(threads)  # each worker's peers live in its own heap arena (batch.cpp ob_rehome)
    G = topo.G
    msgs = np.zeros(0, abi.MESSAGE)
    for k in range(2):  # to steady state
        o = pop.step(msgs, locals_fn(k, pop), threads=threads)
        msgs = topo.route_messages(o["msgs"])
        pop.commit_all(threads)
    passes, t_step, commits = 0, 0.0, 0
    t_end = time.time() + seconds
    k = 2
    while time.time() < t_end or passes < 2:
        if inject is not None:
            inject(k, pop)
        loc = locals_fn(k, pop)
        before = pop.export()["committed"]
        t0 = time.perf_counter()
        o = pop.step(msgs, loc, threads=threads, want_mid=False)  # the raft step only, no record export
        t_step += time.perf_counter() - t0
        end = pop.export()
        commits += int(np.sum((end["committed"] > before) & (end["state"] == abi.LEADER)))
        msgs = topo.route_messages(o["msgs"])
        if drop is not None:
            msgs = drop(k, msgs)
        pop.commit_all(threads)
        passes += 1
        k += 1
    return commits / t_step, G * passes / t_step, passes


def cgroup_cpu_max():
    """The container's CPU quota (cgroup v2 cpu.max, "quota period"), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            return f.read().strip()
    except OSError:
        return None


def effective_cpus(info):
    """CPUs the baseline's threads can actually use: the affinity set, capped by
    the cgroup quota (cpu.max "quota period" -> ceil(quota / period))."""
    n = info.get("affinity_cpus") or info.get("nproc") or 1
    q = info.get("cgroup_cpu_max")
    if q:
        parts = q.split()
        if len(parts) == 2 and parts[0] != "max":
            try:
                n = min(n, max(1, -(-int(parts[0]) // int(parts[1]))))
            except ValueError:
                pass
    return n


def thread_row(nproc):
    """Thread counts of the scaling row: powers of two up to nproc, and nproc."""
    row, t = [], 1
    while t < nproc:
        row.append(t)
        t *= 2
    return row + [nproc]


def cpu_baseline(args, R):
    """BASELINE.md's CPU protocol on bounded samples, host cores only: the oracle
    (C++ restatement of the reference Go step, kind "port") on BASELINE config 4's
    shape (the headline's twin) at T = nproc threads, with a
    thread-scaling row from 1 thread up to nproc, plus configs 2, 3 and 5 on the
    same generators and seeds as the GPU runs at the row's best thread count."""
    import numpy as np
    from dragonboat_amd import abi, populations as P
    info = cpu_info()
    info["cgroup_cpu_max"] = cgroup_cpu_max()
    nproc = info["nproc"] or 1
    eff = effective_cpus(info)
    info["effective_cpus"] = eff
    # the thread row runs up to BASELINE.md's T = nproc; the reported value is the
    # row's best (the strongest CPU number), and `cores` the CPUs those threads
    # could actually use: the threads, capped by the affinity set and the cgroup
    # quota (more threads than that only time-slice the quota's CPU time)
    T = args.cpu_threads or nproc
    G = args.cpu_groups
    budget = args.cpu_seconds
    steady = lambda G_: (lambda k, pop: P.propose_locals(R * G_, np.arange(G_), pass_index=k))
    # config 4's shape (1M x 3 on the GPU): a G-group sample at each thread count
    row = thread_row(T)
    per = 0.5 * budget / len(row)
    scaling = []
    for t in row:
        c, _, n = _oracle_rate(P.make_groups(G, R, seed=2), P.Topology(G, R), R, steady(G), t, per)
        scaling.append({"threads": t, "commits_per_s": c, "passes": n})
    best = max(scaling, key=lambda x: x["commits_per_s"])
    bt = best["threads"]
    out = {"value": best["commits_per_s"], "unit": "commit-index updates/s", "cores": min(bt, eff),
           "threads": bt, "kind": "port",
           "sample": f"config 4 shape: {G} groups x {R} replicas, {best['passes']} passes, oracle raft step "
                     f"timed (message routing and persistence excluded), best of the thread row 1..{T}: "
                     f"{bt} threads on {min(bt, eff)} effective CPUs (nproc {nproc}, cgroup quota "
                     f"{info['cgroup_cpu_max']})",
           "at_nproc": scaling[-1],
           "one_thread": {"value": scaling[0]["commits_per_s"], "passes": scaling[0]["passes"]},
           "best": best, "thread_scaling": scaling,
           "note": "value = the best point of the thread row (1, 2, 4, ... nproc threads); cores = that row's "
                   "threads capped by the affinity set and the cgroup quota (cgroup_cpu_max, ceil(quota/period) "
                   "CPUs): the CPU time the threads can actually get; nproc and effective_cpus are beside it",
           "label": "C++ restatement of reference Go step (oracle/raft_oracle.hpp), not Go",
           **info}
    T = best["threads"]  # the other configs at the row's best thread count
    budget = budget * 0.5
    cfg = {}
    # config 2: 10k x 3 at full size
    G2 = 10_000
    c2, _, n2 = _oracle_rate(P.make_groups(G2, 3, seed=2), P.Topology(G2, 3), 3, steady(G2), T, 0.15 * budget)
    cfg["2"] = {"commits_per_s": c2, "groups": G2, "passes": n2, "threads": T}
    # config 3: 100k x 5, 90% quiesced, ReadIndex + ticks (sample of the same generator)
    G3 = min(20_000, 100_000)
    p3, act3 = P.config3(G3, 5)
    rng3 = np.random.default_rng(3)
    _, g3, n3 = _oracle_rate(p3, P.Topology(G3, 5), 5, lambda k, pop: P.config3_locals(G3, 5, act3, k), T,
                             0.15 * budget, drop=lambda k, m: P.drop_acks(m, 0.1, rng3))
    cfg["3"] = {"groups_per_s": g3, "groups": G3, "passes": n3, "threads": T,
                "sample": f"{G3} of 100k groups x 5 (same generator)"}
    # config 5: leader churn p = 0.1, 100k x 3 (sample)
    G5 = min(20_000, 100_000)
    t5 = P.Topology(G5, 3)
    rng5 = np.random.default_rng(5)

    def inject5(k, pop):
        cur = pop.export()
        ch = P.inject_leader_change(cur, t5, 0.1, rng5)
        if len(ch):
            pop.reload(ch, cur[ch])
    c5, g5, n5 = _oracle_rate(P.make_groups(G5, 3, seed=5), t5, 3,
                              lambda k, pop: P.propose_locals(3 * G5, P.current_leaders(pop.export(), t5),
                                                              pass_index=k),
                              T, 0.15 * budget, inject=inject5)
    cfg["5"] = {"commits_per_s": c5, "groups_per_s": g5, "groups": G5, "passes": n5, "threads": T,
                "sample": f"{G5} of 100k groups x 3 (same generator)"}
    out["configs"] = cfg
    return out


def host_path(args, R, ordinal):
    """The C-ABI path a Go step worker calls (gr_step: host records in, device
    passes, host records out), PCIe-inclusive, at the headline shape. Routing of
    the previous outbox to the receivers (the transport's role) is untimed."""
    import ctypes
    import numpy as np
    from dragonboat_amd import abi, populations as P
    from dragonboat_amd.engine import Engine
    G = args.groups
    peers = P.make_groups(G, R, seed=2)
    topo = P.Topology(G, R)
    eng = Engine(R * G, R, device=ordinal)
    eng.load(peers)
    msgs = np.zeros(0, abi.MESSAGE)
    t_step = 0.0
    n_in = n_out = 0
    warm, passes = 2, args.host_passes
    for k in range(warm + passes):
        loc = P.propose_locals(R * G, np.arange(G), pass_index=k)
        if k == warm:
            eng.reset_stats()
        ib = abi.inbox_of(msgs, loc)
        ob = abi.Outbox()
        t0 = time.perf_counter()
        rc = eng.lib.gr_step(eng._h, ctypes.byref(ib), ctypes.byref(ob))
        t1 = time.perf_counter()
        assert rc == 0, rc
        out = np.zeros(ob.n_msgs, abi.MESSAGE)
        if ob.n_msgs:
            ctypes.memmove(out.ctypes.data, ob.msgs, ob.n_msgs * abi.MESSAGE.itemsize)
        eng.lib.gr_release_outbox(eng._h, ctypes.byref(ob))
        if k >= warm:
            t_step += t1 - t0
            n_in += len(msgs)
            n_out += len(out)
        msgs = topo.route_unsorted(out)
    st = eng.stats()
    eng.close()
    full = {"path": "gr_step: host gr_message/gr_local_input records in, gr_message/gr_peer_result records "
                    "out (PCIe-inclusive)",
            "groups": G, "replicas": R, "passes": passes, "ms_per_pass": t_step / passes * 1e3,
            "commits_per_s": st["leader_commits"] / t_step, "escalations": st["escalations"],
            "msgs_in_per_pass": n_in / passes, "msgs_out_per_pass": n_out / passes,
            "record_bytes_per_pass": (n_in + n_out) / passes * abi.MESSAGE.itemsize
            + R * G * abi.RESULT.itemsize}
    compact = host_path_compact(args, R, ordinal)
    piped = host_path_compact(args, R, ordinal, partitions=args.host_pipeline_partitions, pipelined=True)
    best = piped if piped["ms_per_pass"] < compact["ms_per_pass"] else compact
    return {**best, "other_compact": compact if best is piped else piped, "full_records": full}


def host_path_compact(args, R, ordinal, partitions=None, pipelined=False):
    """gr_step_compact (24-B messages, 40-B results, ext records for the rest):
    the headline shape through the C-ABI, PCIe-inclusive, the way dragonboat's
    step workers would call it (SURVEY.md §8b threading): the groups are split
    clusterID % P over P partitions, each with its own engine (stream, pinned
    inbox/outbox) and its own host thread, and every round the P workers call
    gr_step_compact concurrently, so one partition's upload overlaps another's
    download. The host writes each inbox into the engine's pinned buffers
    (gr_cinbox_reserve), as a Go packer would; routing the previous outbox
    (the transport's role) runs between rounds and is untimed."""
    import ctypes
    import threading
    import numpy as np
    from dragonboat_amd import abi, populations as P
    from dragonboat_amd.engine import Engine
    P_ = partitions or args.host_partitions
    G = args.groups
    sizes = [G // P_ + (1 if w < G % P_ else 0) for w in range(P_)]
    parts = []
    for w, Gw in enumerate(sizes):
        eng = Engine(R * Gw, R, device=ordinal)
        eng.load(P.make_groups(Gw, R, seed=2 + 7919 * w))
        parts.append({"eng": eng, "G": Gw, "topo": P.Topology(Gw, R), "cm": np.zeros(0, abi.CMSG),
                      "cx": np.zeros(0, abi.MESSAGE), "rc": 0, "n_rx": 0})
    warm, passes = 4, args.host_passes  # warm-up grows every pinned buffer to its steady size

    def call(pt):
        pt["ob"] = abi.COutbox()
        pt["rc"] = pt["eng"].lib.gr_step_compact(pt["eng"]._h, ctypes.byref(pt["ib"]), ctypes.byref(pt["ob"]))

    def end(pt):
        pt["ob"] = abi.COutbox()
        pt["rc"] = pt["rc"] or pt["eng"].lib.gr_step_compact_end(pt["eng"]._h, ctypes.byref(pt["ob"]))

    t_step = 0.0
    n_in = n_out = n_x = 0
    for k in range(warm + passes):
        for pt in parts:  # untimed: the host packs each partition's inbox in place
            eng = pt["eng"]
            cl, clx = eng.pack_locals(P.propose_locals(R * pt["G"], np.arange(pt["G"]), pass_index=k))
            if k == warm:
                eng.reset_stats()
            ib = abi.CInbox()
            assert eng.lib.gr_cinbox_reserve(eng._h, len(pt["cm"]), len(pt["cx"]), len(cl), len(clx),
                                             ctypes.byref(ib)) == 0
            for ptr, a in ((ib.msgs, pt["cm"]), (ib.ext_msgs, pt["cx"]), (ib.locals, cl), (ib.ext_locals, clx)):
                if len(a):
                    ctypes.memmove(ptr, a.ctypes.data, a.nbytes)
            pt["ib"] = ib
        t0 = time.perf_counter()
        if pipelined:
            # the uploads one after another (gr_step_compact_begin returns when its
            # copy is done), each partition's pass and download on its own thread
            # meanwhile: PCIe is full duplex, so one partition's download overlaps
            # the next one's upload
            ths = []
            for pt in parts:
                pt["rc"] = pt["eng"].lib.gr_step_compact_begin(pt["eng"]._h, ctypes.byref(pt["ib"]))
                th = threading.Thread(target=end, args=(pt,))
                th.start()
                ths.append(th)
        else:
            ths = [threading.Thread(target=call, args=(pt,)) for pt in parts]
            for th in ths:
                th.start()
        for th in ths:
            th.join()
        t1 = time.perf_counter()
        for pt in parts:
            assert pt["rc"] == 0, pt["rc"]
            ob = pt["ob"]
            om = np.zeros(ob.n_msgs, abi.CMSG)
            ox = np.zeros(ob.n_ext_msgs, abi.MESSAGE)
            if ob.n_msgs:
                ctypes.memmove(om.ctypes.data, ob.msgs, om.nbytes)
            if ob.n_ext_msgs:
                ctypes.memmove(ox.ctypes.data, ob.ext_msgs, ox.nbytes)
            if k >= warm:
                n_in += len(pt["cm"])
                n_out += len(om)
                n_x += len(pt["cx"]) + len(ox) + ob.n_ext_results
            pt["eng"].lib.gr_release_coutbox(pt["eng"]._h, ctypes.byref(ob))
            pt["cm"], pt["cx"] = pt["topo"].route_unsorted(om), pt["topo"].route_unsorted(ox)
        if k >= warm:
            t_step += t1 - t0
    commits = esc = 0
    for pt in parts:
        st = pt["eng"].stats()
        commits += st["leader_commits"]
        esc += st["escalations"]
        pt["eng"].close()
    how = ("pipelined: uploads in turn (gr_step_compact_begin), each partition's pass + download on its own "
           "thread (gr_step_compact_end)" if pipelined else "concurrent step workers")
    return {"path": "gr_step_compact: host gr_cmsg/gr_clocal records in, gr_cmsg/gr_cresult records out "
                    "(+ ext records), PCIe-inclusive, pinned inbox, %d partitions, %s" % (P_, how),
            "groups": G, "replicas": R, "partitions": P_, "passes": passes, "ms_per_pass": t_step / passes * 1e3,
            "commits_per_s": commits / t_step, "escalations": esc,
            "msgs_in_per_pass": n_in / passes, "msgs_out_per_pass": n_out / passes,
            "ext_records_per_pass": n_x / passes,
            "record_bytes_per_pass": (n_in + n_out) / passes * abi.CMSG.itemsize
            + R * G * abi.CRESULT.itemsize + G * abi.CLOCAL.itemsize}


def copy_peak_gbs():
    """Achievable HBM bandwidth on this box: tools/hbm_calib's float4 copy
    (MI355X_MICROARCH.md's 6.29 TB/s method), run as a child process."""
    import subprocess
    exe = os.path.join(ROOT, "tools", "hbm_calib")
    try:
        p = subprocess.run([exe, "copy"], capture_output=True, text=True, timeout=120)
        return json.loads(p.stdout.strip().splitlines()[-1])["copy_f4_GBs"]
    except Exception:
        return None


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
    # GR_BENCH_COLLECTIVE=1 (measurement, not the driver's): with one rank and
    # --placement spread, a one-rank RCCL group moves the exchange buffers with
    # the async all_to_all_single an N > 1 run issues (Exchange(collective=True)),
    # so the N = 8 exchange path's device cost is timed on one GPU
    collective = os.environ.get("GR_BENCH_COLLECTIVE") == "1"
    if world > 1 or collective:
        if world == 1:
            for k_, v_ in (("RANK", "0"), ("WORLD_SIZE", "1"), ("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29531")):
                os.environ.setdefault(k_, v_)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from dragonboat_amd import abi, populations as P
    from dragonboat_amd.engine import Engine
    from dragonboat_amd.exchange import Pipeline

    R = args.replicas
    S = R
    G = args.groups
    # N > 1: BASELINE config 4 (replicas on distinct GPUs, RCCL all-to-all per pass)
    placement = args.placement or ("spread" if world > 1 else "local")
    codec = os.environ.get("GR_BENCH_CODEC", "cx")  # the spread exchange's form (exchange.py)
    pipe = Pipeline(G, R, S, world, rank, placement, banks=args.banks, codec=codec, collective=collective or None)
    pipe.setup(Engine, dev, ordinal)

    for k in range(args.warmup):
        pipe.step(k)
    k0 = args.warmup
    use_graph = args.launch == "graph" and pipe.graph_ready() and args.steps % 2 == 0
    if use_graph:  # untimed: align to the captured pair (it starts in space 0), capture, one warm replay
        if k0 % 2:
            pipe.step(k0)
            k0 += 1
        pipe.graph_steps(k0, 2)
        k0 += 2
    pipe.synchronize()
    if world > 1:
        dist.barrier()
    pipe.reset_stats()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    if use_graph:
        pipe.graph_steps(k0, args.steps)
    else:
        for k in range(args.steps):
            pipe.step(k0 + k)
    pipe.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    st = pipe.stats()
    # Per-kernel durations for the roofline: the same passes once more, outside the
    # timed region, with HIP events around each kernel (recorded inside the library
    # on the bank's stream), so the events add nothing to `value`.
    pipe.timing_begin()
    for k in range(args.steps):
        pipe.step(k0 + args.steps + k)
    pipe.synchronize()
    tm = pipe.timing_end()
    xbytes = pipe.exchange_bytes_per_pass()
    xbytes_heavy = pipe.exchange_bytes_per_pass(heavy=True)
    banks = len(pipe.ex)
    pipe.close()
    commits = st["leader_commits"]
    esc = st["escalations"]
    if world > 1:
        t = torch.tensor([commits, esc], dtype=torch.float64, device=cdev)
        dist.all_reduce(t)
        commits, esc = int(t[0].item()), int(t[1].item())
    value = commits / elapsed
    passes = max(1, tm["passes"])
    kavg = tm["fast_ms"] / passes  # the dominant kernel, HIP events on the pass's stream
    gavg = tm["general_ms"] / passes
    groups_total = G * world
    # SURVEY.md §8d's unit: one group-round (R-1 acks in, quorum commit, R-1
    # Replicates out, R-1 follower matches) = B_round(R) bytes at reference field
    # widths; a launch processes one group-round per leader commit.
    rounds = st["leader_commits"] / (args.steps * banks)  # per launch (one bank's pass)
    canon = b_round(R) * rounds  # SURVEY.md 8d canonical bytes per launch (reference widths)
    canon_achieved = canon / (kavg * 1e-3) / 1e9
    alg = ENCODED_ROUND_BYTES.get(R, b_round(R)) * rounds  # algorithmic bytes per launch (this rank)
    achieved = alg / (kavg * 1e-3) / 1e9
    refw = reference_width_bytes(st, G, R, args.steps) / (args.steps * banks)
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
        copy_gbs = copy_peak_gbs()
        traffic_gbs = traffic / (kavg * 1e-3) / 1e9 if traffic else None
        configs_ev = None  # BASELINE configs 2, 3, 5 on this build (tools/configs_summary.py), never `value`
        cfg_path = os.path.join(ROOT, "profiles", "configs_latest.json")
        if os.path.exists(cfg_path):
            try:
                from dragonboat_amd.build import source_digest
                rec = json.load(open(cfg_path))
                if rec.get("source_digest") == source_digest():
                    configs_ev = {k: {f: v.get(f) for f in ("config", "device_ms_per_pass", "stream_ms_per_pass",
                                                              "pmc_bytes_per_pass", "canonical_bytes_per_pass",
                                                              "pmc_over_canonical", "canonical_frac")}
                                  for k, v in rec.get("configs", {}).items()}
                    configs_ev["source"] = "profiles/configs_latest.json (same source digest as this build)"
            except (OSError, ValueError):
                configs_ev = None
        try:  # provenance: the loaded library's build record against this tree's sources
            from dragonboat_amd.build import build_record, source_digest
            brec = build_record(os.environ.get("GPURAFT_LIB") or None) or {}
            build_info = {"lib": brec.get("lib"), "built_from": brec.get("source_digest"),
                          "tree": source_digest(), "built_at": brec.get("built_at"),
                          "compiler": brec.get("compiler")}
            build_info["matches_tree"] = build_info["built_from"] == build_info["tree"]
        except Exception:  # the record is informational; never fail the bench over it
            build_info = None
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
                       "replicas": R, "placement": placement, "banks": banks,
                       "parallelism": f"clusterID shards x{world}" + (", replicas on distinct GPUs, RCCL "
                                                                    "all_to_all per pass" if placement == "spread"
                                                                    else "")},
            "launch": "graph (gr_graph_replay of a captured two-pass graph)" if use_graph else "stream (kernel launches)",
            "escalations": esc,
            "exchange_bytes_per_pass": xbytes,
            "exchange_bytes_heavy_pass": xbytes_heavy,
            "exchange_codec": codec if placement == "spread" and (world > 1 or collective) else None,
            "exchange_collective": "RCCL all_to_all_single, async on the bank's stream" + (
                " (one-rank rehearsal: GR_BENCH_COLLECTIVE=1)" if world == 1 else "")
            if placement == "spread" and (world > 1 or collective) else None,
            "build": build_info,
            "configs_evidence": configs_ev,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": f"lean kernels of one pass (gr_steady_kernel<{S},{R}>; gr_roles_kernel<{S},{R}> too on a pass "
                                   "whose tail plan launches the role instances, none in the steady state)",
                         "kernel_ms": kavg,
                         "algorithmic_bytes_per_launch": alg,
                         "algorithmic_unit": (f"group-round at this engine's encoding, {ENCODED_ROUND_BYTES[R]} B "
                                              "(bench.py ENCODED_ROUND_BYTES, DESIGN.md 3)" if R in ENCODED_ROUND_BYTES
                                              else f"group-round, B_round({R}) = {b_round(R)} B (SURVEY.md 8d)"),
                         "canonical_bytes_per_launch": canon,
                         "canonical_unit": f"group-round, B_round({R}) = {b_round(R)} B (SURVEY.md 8d, reference "
                                           "field widths: more bytes than the kernels move)",
                         "canonical_achieved": canon_achieved,
                         "canonical_frac": canon_achieved / HBM_PEAK_GBS,
                         "group_rounds_per_launch": rounds,
                         "traffic_GBs": traffic_gbs,
                         "traffic_frac": traffic_gbs / HBM_PEAK_GBS if traffic else None,
                         "copy_f4_GBs": copy_gbs,
                         "traffic_frac_of_copy": traffic_gbs / copy_gbs if traffic and copy_gbs else None,
                         "reference_width_bytes_per_launch": refw,
                         "reference_width_note": "two Replicates + two acks per follower per round at "
                                                 "reference field widths (1,128 B/group): never used as frac",
                         "general_kernel_ms": gavg,
                         "bailed_lanes_per_pass": tm["bailed_lanes"] / passes},
        }
        if args.host_path == "on" and world == 1:
            try:
                line["host_path"] = host_path(args, R, ordinal)
            except Exception as e:  # reported beside the headline, never as `value`
                line["host_path"] = {"error": str(e)}
        if args.cpu_baseline == "on" and world == 1:
            try:
                line["cpu_baseline"] = cpu_baseline(args, R)
            except Exception as e:  # baseline is reported, not required
                line["cpu_baseline"] = {"value": None, "error": str(e)}
        print(json.dumps(line), flush=True)
    if world > 1 or collective:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
