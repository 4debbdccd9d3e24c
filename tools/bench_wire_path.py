"""The wire path at the headline shape (1M groups x 3, steady state): MessageBatch
frames uploaded, decoded in HBM (libgrwire) and routed straight into the step
pass (gr_step_wire), next to gr_step with the same messages as host records.

Per pass, timed (wall clock): frame upload + grw_decode_device + gr_step_wire
(which downloads the outbox records and results). Untimed: building the frames
the senders' transports would send (tests/wirefeed.py) from the previous pass's
outbox. Prints one JSON line.

    python tools/bench_wire_path.py --groups 1000000 --passes 3
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=1_000_000)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--compact", action="store_true", help="gr_step_wire_compact (24-B outbox records)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from dragonboat_amd import abi, populations as P, wire as W
    from dragonboat_amd.engine import Engine
    import wirefeed
    G, R = a.groups, 3
    n = R * G
    peers = P.make_groups(G, R, seed=2)
    topo = P.Topology(G, R)
    cl = (np.arange(n) % G) + 1
    eng = Engine(n, R)
    eng.load(peers)
    eng.bind_nodes(cl, peers["node_id"])
    codec = W.WireCodec(0)
    msgs = np.zeros(0, abi.MESSAGE)
    t_up = t_dec = t_step = 0.0
    frame_bytes = nmsg = 0
    for k in range(a.warmup + a.passes):
        loc = P.propose_locals(n, np.arange(G), pass_index=k)
        batches, wm, we, payload = wirefeed.to_wire(msgs, peers["node_id"], peers["remote_id"], cl, per_frame=256)
        frames = codec.marshal(payload, batches, wm, we) if len(wm) else np.zeros(0, np.uint8)
        table = W.frames_table(batches["frame_off"], batches["frame_len"])
        if k == a.warmup:
            eng.reset_stats()
        h_buf = torch.from_numpy(frames).pin_memory() if len(wm) else None  # the transport's pass buffer
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if len(wm):
            d_buf = h_buf.cuda(non_blocking=True)
            d_bat = torch.from_numpy(table.view(np.uint8)).cuda()
            d_msgs = torch.empty(len(wm) * W.WMESSAGE.itemsize, dtype=torch.uint8, device="cuda")
            d_ents = torch.empty(max(1, len(we)) * W.WENTRY.itemsize, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            nm, ne = codec.unmarshal_device(d_buf.data_ptr(), len(frames), d_bat.data_ptr(), len(table),
                                            d_msgs.data_ptr(), len(wm), d_ents.data_ptr(), max(1, len(we)))
            t2 = time.perf_counter()
            # the C-ABI call a Go step worker makes; its outbox is engine-owned pinned
            # memory the caller reads in place (the copy into numpy below is untimed)
            import ctypes
            ob, un = (abi.COutbox() if a.compact else abi.Outbox()), abi.WireUnrouted()
            loc_c = np.ascontiguousarray(loc, abi.LOCAL)
            fn = eng.lib.gr_step_wire_compact if a.compact else eng.lib.gr_step_wire
            rc = fn(eng._h, d_msgs.data_ptr(), nm, d_ents.data_ptr(), ne, loc_c.ctypes.data, len(loc_c),
                    ctypes.byref(ob), ctypes.byref(un))
            t3w = time.perf_counter()
            assert rc == 0 and un.n == 0, (rc, un.n)
            if a.compact:  # the next pass's inbox: the compact records expanded (untimed)
                cm, xm, _, _ = eng._take_coutbox(ob)
                out = eng.unpack_messages(cm, xm)
            else:
                out = np.zeros(ob.n_msgs, abi.MESSAGE)
                ctypes.memmove(out.ctypes.data, ob.msgs, ob.n_msgs * abi.MESSAGE.itemsize)
                eng.lib.gr_release_outbox(eng._h, ctypes.byref(ob))
        else:
            t1 = t2 = time.perf_counter()
            out, res = eng.step(msgs, loc)
            t3w = time.perf_counter()
        t3 = t3w
        if k >= a.warmup:
            t_up += t1 - t0
            t_dec += t2 - t1
            t_step += t3 - t2
            frame_bytes += len(frames)
            nmsg += len(wm)
        msgs = topo.route_messages(out)
    st = eng.stats()
    codec.close()
    eng.close()
    p = a.passes
    print(json.dumps({
        "path": ("gr_step_wire_compact" if a.compact else "gr_step_wire") +
                ": MessageBatch frames uploaded, decoded in HBM (grw_decode_device), routed into the step pass; "
                "outbox " + ("compact gr_cmsg/gr_cresult" if a.compact else "gr_message/gr_peer_result") +
                " records downloaded into engine-owned pinned memory (the caller reads them in place; copying "
                "them out is not timed)",
        "groups": G, "replicas": R, "passes": p,
        "ms_per_pass": (t_up + t_dec + t_step) / p * 1e3,
        "upload_ms": t_up / p * 1e3, "decode_ms": t_dec / p * 1e3, "route_step_download_ms": t_step / p * 1e3,
        "frame_bytes_per_pass": frame_bytes / p, "msgs_per_pass": nmsg / p,
        "commits_per_s": st["leader_commits"] / (t_up + t_dec + t_step)}), flush=True)


if __name__ == "__main__":
    main()
