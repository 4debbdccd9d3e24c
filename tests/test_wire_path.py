"""The wire path (SURVEY.md §8f-2 feeding the inbox): MessageBatch frames are the
only inbox bytes that cross PCIe; libgrwire decodes them in HBM and gr_step_wire
routes the decoded raftpb.Message records into the pass (gpuraft.h). Checked
against the oracle after every pass with the same Lockstep the other backends
use, and against the reasons a message stays with the host."""
import numpy as np
import pytest

from dragonboat_amd import abi, populations as P, wire as W
import simulate as SIM

pytestmark = pytest.mark.gpu


def test_wire_path_churn(gpu):
    """BASELINE config 5's shape: leader changes with divergent suffixes (rejects,
    truncations, multi-entry catch-up Replicates, forwarded proposals)."""
    G, R = 400, 3
    topo = P.Topology(G, R)
    rng = np.random.default_rng(5)
    st = SIM.simulate(SIM.GpuWireBackend, P.make_groups(G, R, seed=5), topo, 12,
                      lambda k, s: P.propose_locals(R * G, P.current_leaders(s, topo), pass_index=k),
                      inject_fn=lambda k, cur: P.inject_leader_change(cur, topo, 0.1, rng))
    assert st["commits"] > 0 and st["msgs"] > 0


def test_wire_path_ticks_read_index(gpu):
    """Heartbeats with ReadIndex contexts, their acks, CheckQuorum (config 3's
    message kinds) through frames, R = 5."""
    G, R = 200, 5
    peers, active = P.config3(G, R)
    rng = np.random.default_rng(3)
    st = SIM.simulate(SIM.GpuWireBackend, peers, P.Topology(G, R), 8, lambda k: P.config3_locals(G, R, active, k),
                      slots=5, drop_fn=lambda k, m: P.drop_acks(m, 0.1, rng))
    assert st["ready"] > 0


def test_wire_compact_at_scale_churn_heartbeats(gpu):
    """gr_step_wire_compact (frames in, compact records out) at BASELINE config 5's
    size, 100k x 3, against the oracle after every pass: leader changes with
    p = 0.1 from the second pass (step-downs, term adoptions, rejects, truncations,
    multi-entry catch-ups), and a Tick on every replica every third pass (leader
    heartbeats and their acks: full records through the codec and back)."""
    G, R = 100_000, 3
    topo = P.Topology(G, R)
    rng = np.random.default_rng(55)

    def locals_fn(k, s):
        return P.propose_locals(R * G, P.current_leaders(s, topo), pass_index=k, ticks=1 if k % 3 == 2 else 0)
    st = SIM.simulate(SIM.GpuWireCompactBackend, P.make_groups(G, R, seed=55), topo, 6, locals_fn,
                      inject_fn=lambda k, cur: P.inject_leader_change(cur, topo, 0.1, rng) if k >= 1 else None)
    assert st["commits"] > 0 and st["msgs"] > 3 * G


def test_wire_unrouted_reasons(gpu):
    """Messages the device cannot step stay with the host, each with its reason;
    the others step exactly as gr_step steps the same records."""
    import torch
    import wirefeed
    from dragonboat_amd.engine import Engine
    G, R = 64, 3
    peers = P.make_groups(G, R, seed=2)
    topo = P.Topology(G, R)
    cl = (np.arange(R * G) % G) + 1
    # one steady pass's messages (the oracle's routing of a first pass)
    from oracle.pyoracle import OraclePopulation
    pop = OraclePopulation(peers, R)
    o = pop.step(np.zeros(0, abi.MESSAGE), P.propose_locals(R * G, np.arange(G), pass_index=0))
    msgs = topo.route_messages(o["msgs"])
    assert len(msgs) > 8
    batches, wm, we, payload = wirefeed.to_wire(msgs, peers["node_id"], peers["remote_id"], cl)
    n = len(wm)
    # corrupt five messages, one per reason
    bad = {0: "no_peer", 1: "nonmember", 2: "index", 3: "type", 4: "runs"}
    wm[0]["cluster_id"] = 10**9
    wm[1]["from"] = 999
    rep = np.nonzero((wm["type"] == abi.REPLICATE) & (wm["n_entries"] > 0))[0]
    rep = [int(x) for x in rep if x > 4]
    assert len(rep) >= 2
    # swap message 2 with a Replicate carrying entries, then break its entry indices
    order = np.arange(n)
    order[[2, rep[0]]] = order[[rep[0], 2]]
    order[[4, rep[1]]] = order[[rep[1], 4]]
    wm2, ents = wm[order].copy(), []
    for i in range(n):  # rebuild the entry array in the new message order
        m = wm2[i]
        e = we[int(m["first_entry"]):int(m["first_entry"]) + int(m["n_entries"])].copy()
        if i == 2:
            e["index"] += 5
        if i == 4:  # three term runs
            e = np.concatenate([e, e, e])
            e["term"] = [1, 2, 3][:len(e)] + [3] * max(0, len(e) - 3)
            m["n_entries"] = len(e)
        wm2[i]["first_entry"] = sum(len(x) for x in ents)
        wm2[i]["n_entries"] = len(e)
        ents.append(e)
    we2 = np.concatenate(ents)
    wm2[3]["type"] = 40
    codec = W.WireCodec(0)
    frames = codec.marshal(payload, batches, wm2, we2)
    table = W.frames_table(batches["frame_off"], batches["frame_len"])
    d_buf = torch.from_numpy(frames).cuda()
    d_bat = torch.from_numpy(table.view(np.uint8)).cuda()
    d_msgs = torch.empty(n * W.WMESSAGE.itemsize, dtype=torch.uint8, device="cuda")
    d_ents = torch.empty(len(we2) * W.WENTRY.itemsize, dtype=torch.uint8, device="cuda")
    nm, ne = codec.unmarshal_device(d_buf.data_ptr(), len(frames), d_bat.data_ptr(), len(table), d_msgs.data_ptr(),
                                    n, d_ents.data_ptr(), len(we2))
    codec.close()
    assert nm == n
    loc = P.propose_locals(R * G, np.arange(G), pass_index=1)
    eng = Engine(R * G, R)
    eng.load(peers)
    eng.bind_nodes(cl, peers["node_id"])
    out_w, res_w, idx, why = eng.step_wire(d_msgs.data_ptr(), nm, d_ents.data_ptr(), ne, loc)
    got = {int(i): abi.WIRE_REASONS[int(w)] for i, w in zip(idx, why)}
    assert got == bad, got
    # the routed ones step exactly as gr_step with the same records
    keep = np.array([i for i in range(n) if i not in bad])
    ref = Engine(R * G, R)
    ref.load(peers)
    out_r, res_r = ref.step(msgs[order][keep], loc)
    assert np.array_equal(out_w, out_r) and np.array_equal(res_w, res_r)
    assert np.array_equal(eng.sync(R * G), ref.sync(R * G))
    eng.close()
    ref.close()


def test_wire_compact_outbox(gpu):
    """gr_step_wire_compact returns exactly what gr_step_compact returns for the
    same messages and locals (compact records, ext records, compact results)."""
    import torch
    import wirefeed
    from dragonboat_amd.engine import Engine
    from oracle.pyoracle import OraclePopulation
    G, R = 300, 3
    peers = P.make_groups(G, R, seed=4)
    topo = P.Topology(G, R)
    cl = (np.arange(R * G) % G) + 1
    pop = OraclePopulation(peers, R)
    o = pop.step(np.zeros(0, abi.MESSAGE), P.propose_locals(R * G, np.arange(G), pass_index=0))
    msgs = topo.route_messages(o["msgs"])
    feed = wirefeed.WireFeed(peers, cl)
    d_m, nm, d_e, ne, keep = feed.decode(msgs)
    loc = P.propose_locals(R * G, np.arange(G), pass_index=1)
    loc["ticks"][::7] = 1
    eng = Engine(R * G, R)
    eng.load(peers)
    eng.bind_nodes(cl, peers["node_id"])
    got, idx, why = eng.step_wire(d_m, nm, d_e, ne, loc, compact=True)
    feed.close()
    assert len(idx) == 0
    ref = Engine(R * G, R)
    ref.load(peers)
    cm, xm = ref.pack_messages(msgs)
    cloc, xloc = ref.pack_locals(loc)
    want = ref.step_compact(cm, xm, cloc, xloc)
    for a, b in zip(got, want):
        assert a.dtype == b.dtype and np.array_equal(a, b)
    assert len(got[0]) > 0
    assert np.array_equal(eng.sync(R * G), ref.sync(R * G))
    eng.close()
    ref.close()
    del keep, torch
