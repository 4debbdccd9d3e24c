"""The drop-in boundary's own rate: gr_step (include/gpuraft.h) with host-side
gr_message / gr_local_input arrays in and gr_message / gr_peer_result arrays
out, as the Go step worker would call it, one MI355X.

Each pass: the previous pass's outbox is routed to receivers on the host
(populations.Topology.route_messages, the transport's role, NOT timed), then
gr_step runs: inbox packing, upload, the two kernels, download and outbox
unpacking (timed, wall clock). Kernel time comes from gr_timing (HIP events),
so host+PCIe overhead = step - kernels.

Usage: python tools/bench_host_path.py [--groups G] [--passes N] > gpurun_out/host_path.json
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=1_000_000)
    ap.add_argument("--replicas", type=int, default=3)
    ap.add_argument("--passes", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pinned", action="store_true", help="fill a gr_inbox_reserve buffer instead of passing pageable arrays")
    args = ap.parse_args()
    import numpy as np
    import torch
    torch.cuda.set_device(0)
    from dragonboat_amd import abi, populations as P
    from dragonboat_amd.engine import Engine

    G, R = args.groups, args.replicas
    peers = P.make_groups(G, R, seed=2)
    topo = P.Topology(G, R)
    eng = Engine(R * G, R)
    eng.load(peers)
    msgs = np.zeros(0, abi.MESSAGE)
    t_step = t_kern = 0.0
    n_in = n_out = commits = 0
    for k in range(args.warmup + args.passes):
        loc = P.propose_locals(R * G, np.arange(G), pass_index=k)
        timed = k >= args.warmup
        if k == args.warmup:
            eng.reset_stats()
        if timed:
            eng.timing_begin()
        # the C-ABI call alone (what a Go step worker pays), then a copy out
        msgs = np.ascontiguousarray(msgs, abi.MESSAGE)  # alive across the call
        if args.pinned:  # records written in place into engine-owned pinned memory (untimed)
            ib, mv, lv = eng.reserve_inbox(len(msgs), len(loc))
            mv[:] = msgs
            lv[:] = loc
        else:
            ib = abi.inbox_of(msgs, loc)
        ob = abi.Outbox()
        t0 = time.perf_counter()
        rc = eng.lib.gr_step(eng._h, ctypes.byref(ib), ctypes.byref(ob))
        t1 = time.perf_counter()
        assert rc == 0, rc
        out = np.zeros(ob.n_msgs, abi.MESSAGE)
        res = np.zeros(ob.n_results, abi.RESULT)
        if ob.n_msgs:
            ctypes.memmove(out.ctypes.data, ob.msgs, ob.n_msgs * abi.MESSAGE.itemsize)
        ctypes.memmove(res.ctypes.data, ob.results, ob.n_results * abi.RESULT.itemsize)
        eng.lib.gr_release_outbox(eng._h, ctypes.byref(ob))
        if timed:
            tm = eng.timing_end()
            t_step += t1 - t0
            t_kern += (tm["fast_ms"] + tm["general_ms"]) * 1e-3
            n_in += len(msgs)
            n_out += len(out)
            assert not np.any(res["escalation"]), "escalation in the steady state"
        msgs = topo.route_messages(out)
    st = eng.stats()
    passes = args.passes
    line = {
        "path": "gr_step (host arrays in/out, PCIe-inclusive)" + (", pinned inbox" if args.pinned else ""),
        "groups": G, "replicas": R, "passes": passes,
        "ms_per_pass": t_step / passes * 1e3,
        "kernel_ms_per_pass": t_kern / passes * 1e3,
        "host_and_pcie_ms_per_pass": (t_step - t_kern) / passes * 1e3,
        "msgs_in_per_pass": n_in / passes, "msgs_out_per_pass": n_out / passes,
        "msgs_per_s": (n_in + n_out) / t_step,
        "leader_commits_per_s": st["leader_commits"] / t_step,
        "lib": os.path.basename(os.environ.get("GPURAFT_LIB", "libgpuraft.so")),
    }
    print(json.dumps(line), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
