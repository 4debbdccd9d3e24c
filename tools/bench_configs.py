"""Per-config measurements beside the headline bench (BASELINE.json configs 2, 3, 5)
on one GPU, device-resident path (gr_step_device + mailbox spaces in HBM).

Each pass's host work (new local inputs, config 5's injected leader changes and
reloads) happens outside the timed region; the reported time is the sum of the
two kernels' HIP-event durations per pass (gr_timing), i.e. the device pass. A
device fill queued ahead of each pass hides the CPU launch latency from the events.

  config 2: 10k groups x 3, one 1-entry proposal per leader per pass (replica
            blocks padded to whole waves with idle groups: 10,048 lanes each)
  config 3: 100k groups x 5, 90% quiesced (QuiescedTick), 10% active: a Tick per
            replica and a ReadIndex on the leader per pass (all acks delivered:
            the device path has no drop filter)
  config 5: 100k groups x 3, one proposal per leader per pass, and with p = 0.1
            per group per pass an injected leader change with a divergent
            suffix of 1..8 entries on the old leader (populations.inject_leader_change)
Escalated lanes are counted; the host replay of escalations is not part of
this device measurement (config 5 reloads the changed groups each pass).

Usage: python tools/bench_configs.py [--passes N] > gpurun_out/configs.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(name, peers, G, R, passes, warmup, prepare, graph_reps=0, stream_reps=0):
    """prepare(k, eng, n_peers) -> local inputs of pass k (may also reload groups).
    graph_reps > 0: afterwards, two passes captured with the library's graph mode
    (gr_graph_capture) and replayed graph_reps times (gr_graph_replay): the per-pass
    time with no CPU launch in it. The local inputs then stay
    those of the last pass (config 2's proposals are the same every pass).
    stream_reps > 0: the same passes through gr_step_device, stream_reps of them
    enqueued back to back behind a device sleep (no caller-side graph, no event
    between passes): HIP events around the batch give the per-pass device time,
    perf_counter around the enqueue loop the host's cost per call."""
    import torch
    from dragonboat_amd.engine import Engine
    from dragonboat_amd.exchange import Exchange

    S = R
    ex = Exchange(G, R, S, 1, 0, "local")
    eng = Engine(ex.n_peers, S)
    eng.load(peers)
    eng.bind_routes(ex.in_pos, ex.out_pos)
    spaces = ex.allocate(eng, torch.device("cuda", 0))
    stream = torch.cuda.current_stream()
    fast = gen = 0.0
    bailed = 0
    t_host = 0.0
    # a device fill queued ahead of each timed pass keeps the GPU busy while the
    # CPU launches the pass, so the HIP events time the kernels, not the launch
    pad = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    for k in range(warmup + passes):
        if k == warmup:
            torch.cuda.synchronize()
            eng.reset_stats()
        th = time.perf_counter()
        eng.set_locals(prepare(k, eng, ex.n_peers))
        t_host += time.perf_counter() - th
        if k >= warmup:
            eng.timing_begin()
        pad.fill_(k & 0xFF)
        ex.step(eng, spaces, k, stream)
        if k >= warmup:
            tm = eng.timing_end()
            fast += tm["fast_ms"]
            gen += tm["general_ms"]
            bailed += tm["bailed_lanes"]
    st = eng.stats()
    graph = None
    if graph_reps:
        # the library's graph mode (gr_graph_capture / gr_graph_replay): two passes
        # captured once over the ping-pong spaces, replayed graph_reps times
        if (warmup + passes) & 1:  # the captured pair starts in space 0
            ex.step(eng, spaces, warmup + passes, stream)
        torch.cuda.synchronize()
        g = eng.graph_capture(spaces[0].data_ptr(), spaces[1].data_ptr(), ex.n_chunks, ex.positions, ex.n_peers,
                              n_passes=2, depth=ex.depth)
        eng.graph_replay(g, stream.cuda_stream)  # warm
        torch.cuda.synchronize()
        c0 = eng.stats()["leader_commits"]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(graph_reps):
            eng.graph_replay(g, stream.cuda_stream)
        e1.record()
        torch.cuda.synchronize()
        eng.graph_destroy(g)
        gms = e0.elapsed_time(e1) / (2 * graph_reps)
        commits = eng.stats()["leader_commits"] - c0
        graph = {"api": "gr_graph_capture/gr_graph_replay", "passes": 2 * graph_reps, "ms_per_pass": gms,
                 "leader_commits_per_pass": commits / (2 * graph_reps),
                 "leader_commits_per_s": commits / (2 * graph_reps * gms * 1e-3)}
    stream = None
    if stream_reps:
        k0 = warmup + passes + (2 if graph_reps else 0) + ((warmup + passes) & 1 if graph_reps else 0)
        cs = torch.cuda.current_stream()
        for k in range(k0, k0 + 4):  # warm
            ex.step(eng, spaces, k, cs)
        torch.cuda.synchronize()
        c0 = eng.stats()["leader_commits"]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(2.4e9 * 25e-6 * stream_reps))  # outlasts the host's enqueue loop
        e0.record()
        th = time.perf_counter()
        for k in range(k0 + 4, k0 + 4 + stream_reps):
            ex.step(eng, spaces, k, cs)
        th = time.perf_counter() - th
        e1.record()
        torch.cuda.synchronize()
        sms = e0.elapsed_time(e1) / stream_reps
        commits = eng.stats()["leader_commits"] - c0
        stream = {"api": "gr_step_device, passes enqueued back to back", "passes": stream_reps, "ms_per_pass": sms,
                  "host_enqueue_us_per_pass": th / stream_reps * 1e6,
                  "leader_commits_per_pass": commits / stream_reps,
                  "leader_commits_per_s": commits / (stream_reps * sms * 1e-3)}
    from dragonboat_amd import abi
    import numpy as np
    res = eng.collect_results(ex.n_peers)  # the last pass's per-lane results
    esc = res["escalation"][res["escalation"] != 0]
    reasons = {abi.ESC_NAMES[int(e)]: int(c) for e, c in zip(*np.unique(esc, return_counts=True))}
    ms = (fast + gen) / passes
    out = {"config": name, "groups": G, "replicas": R, "passes": passes,
           "device_ms_per_pass": ms, "fast_ms": fast / passes, "general_ms": gen / passes,
           "bailed_lanes_per_pass": bailed / passes,
           "general_lanes_per_pass": bailed / passes, "lanes": ex.n_peers,
           "lanes_per_s": ex.n_peers / (ms * 1e-3),
           "leader_commits_per_s": st["leader_commits"] / (passes * ms * 1e-3),
           "escalations_per_pass": st["escalations"] / passes,
           "msgs_in_per_pass": st["msgs_in"] / passes, "host_s": t_host,
           "last_pass_escalations": reasons}
    if graph:
        out["graph"] = graph
    if stream:
        out["stream"] = stream
    eng.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--only", default="2,3,5")
    ap.add_argument("--graph-reps", type=int, default=200, help="config 2: replays of a 2-pass HIP graph (0: off)")
    ap.add_argument("--stream-reps", type=int, default=400,
                    help="config 2: gr_step_device passes enqueued back to back (0: off)")
    ap.add_argument("--groups2", type=int, default=10_000, help="config 2's group count")
    ap.add_argument("--align", type=int, default=64, help="config 2: replica blocks padded to this many lanes")
    args = ap.parse_args()
    import numpy as np
    import torch
    torch.cuda.set_device(0)
    from dragonboat_amd import populations as P
    res = []
    want = set(args.only.split(","))
    if "2" in want:
        # replica blocks padded to whole waves (Gl = G rounded up to 64 lanes): the
        # Gl - G padding groups get no input (idle groups, as a host has), so every
        # wave holds lanes of one replica, i.e. one role, and keeps its steady hint;
        # unpadded, the waves straddling the three block boundaries mix leaders and
        # followers, lose the closed forms and set the pass time (A/B: --align 1)
        G, R = args.groups2, 3
        Gl = -(-G // args.align) * args.align
        peers = P.make_groups(Gl, R, seed=2)
        r = run(f"2: {G} x 3, uniform proposals", peers, Gl, R, args.passes, args.warmup,
                lambda k, eng, n: P.propose_locals(n, np.arange(G), pass_index=k), graph_reps=args.graph_reps,
                stream_reps=args.stream_reps)
        r["groups"], r["lane_groups"] = G, Gl
        res.append(r)
    if "3" in want:
        G, R = 100_000, 5
        peers, active = P.config3(G, R)
        res.append(run("3: 100k x 5, 90% quiesced, ReadIndex + ticks", peers, G, R, args.passes,
                       args.warmup, lambda k, eng, n: P.config3_locals(G, R, active, k)))
    if "5" in want:
        G, R = 100_000, 3
        peers = P.make_groups(G, R, seed=5)
        topo = P.Topology(G, R)
        rng = np.random.default_rng(5)

        def prepare5(k, eng, n):
            cur = eng.sync(n)
            if k >= args.warmup and len(P.inject_leader_change(cur, topo, 0.1, rng)):
                eng.load(cur)  # host-side fault injection, reloaded before the pass
            return P.propose_locals(n, P.current_leaders(cur, topo), pass_index=k)
        res.append(run("5: 100k x 3, leader churn p=0.1", peers, G, R, args.passes, args.warmup, prepare5))
    for r in res:
        r["lib"] = os.path.basename(os.environ.get("GPURAFT_LIB", "libgpuraft.so"))
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
