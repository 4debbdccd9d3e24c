"""GPU parity: the HIP kernel (libgpuraft.so through the C-ABI) against the
oracle, bit-exact, on the host-staged path (gr_step) and the device-resident
path (gr_step_device + mailbox spaces)."""
import os

import numpy as np
import pytest

from dragonboat_amd import populations as P
import simulate as SIM

pytestmark = pytest.mark.gpu


def _loaded_native():
    with open("/proc/self/maps") as f:
        return "libgpuraft.so" in f.read()


def test_smoke(gpu):
    import __graft_entry__ as ge
    ge.smoke()
    assert _loaded_native()


def _sim(G, passes, seed, locals_fn=None, inject_p=0.0, **mk):
    R = 3
    peers = P.make_groups(G, R, seed=seed, **mk)
    topo = P.Topology(G, R)
    rng = np.random.default_rng(seed)
    lf = locals_fn or (lambda k: P.propose_locals(R * G, np.arange(G), pass_index=k))
    inj = (lambda k, cur: P.inject_leader_change(cur, topo, inject_p, rng)) if inject_p else None
    return SIM.simulate(SIM.GpuBackend, peers, topo, passes, lf, inject_fn=inj)


def test_gpu_steady_state(gpu):
    st = _sim(1000, 6, seed=3)
    assert st["escalations"] == 0 and st["commits"] > 0


def test_gpu_leader_change_churn(gpu):
    st = _sim(500, 16, seed=5, inject_p=0.1)
    assert st["commits"] > 0


@pytest.mark.parametrize("check_quorum", [False, True])
def test_gpu_ticks_and_read_index(gpu, check_quorum):
    G, R = 256, 3
    rng = np.random.default_rng(9)

    def lf(k):
        loc = P.propose_locals(R * G, np.arange(G), pass_index=k)
        loc["ticks"] = rng.integers(0, 3, R * G)
        loc["read_index"] = rng.random(R * G) < 0.3
        loc["read_ctx_low"] = rng.integers(1, 2**63, R * G, dtype=np.uint64)
        loc["read_ctx_high"] = k
        loc["propose_entries"] = np.where(rng.random(R * G) < 0.5, loc["propose_entries"], 0)
        return loc
    _sim(G, 10, seed=7, locals_fn=lf, check_quorum=check_quorum)


@pytest.mark.parametrize("placement", ["local", "spread"])
def test_device_resident_path(gpu, placement):
    """The bench path: spaces in HBM, routes bound once, locals bound once."""
    import devsim
    final = devsim.run_device(777, 3, 6, placement=placement)
    assert np.all(final["committed"][:777] > 2**32)


@pytest.mark.parametrize("mix", [False, True])
def test_split_pass_churn(gpu, mix, monkeypatch):
    """Large-pass schedule (StepParams::split) forced on a small population, with
    BASELINE config 5's leader changes every pass, checked against the oracle
    after every pass (state, every mailbox, results). mix = False: loopback
    routes, so the steady kernel runs and the role instances walk its wave lists
    while churn puts new leaders into follower-hinted waves; mix = True: peers
    group-major, so every wave holds both roles (unhinted waves through both
    instances, table routes)."""
    import devsim
    monkeypatch.setenv("GR_SPLIT_MIN_LANES", "1")
    monkeypatch.setenv("GR_SMALL_BLOCKS", "0")  # not the fused small-pass kernel
    st = {}
    devsim.run_device(2000, 3, 10, inject_p=0.1, mix=mix, stats=st, seed=11)
    assert st["injected"] > 0


@pytest.mark.parametrize("codec", ["dense", "cx"])
def test_spread_cold_fields_by_side_buffer(gpu, codec):
    """Spread exchange, no host read-back, parity every pass. dense: the hot region
    every pass, the cold fields of the mailboxes that need them (heartbeats and
    their acks, ticks every third pass) through the device-packed side buffers.
    cx (the compact exchange): 12-byte records for the steady mailboxes and,
    round 6, for the tick passes' too (pattern records: a leader's commit
    broadcast, heartbeat and proposal; a follower's acks around its
    HeartbeatResp), so the compact passes carry no full entry at all; every
    fourth pass exchanges the dense form instead (a heavy pass), so the forms
    alternate between passes."""
    import devsim
    st = {}
    cx = codec == "cx"
    final = devsim.run_device(500, 3, 9, placement="spread", tick_every=3, stats=st, codec=codec,
                              heavy_every=4 if cx else 0)
    assert np.all(final["committed"][:500] > 2**32)
    used = [n > 0 for n in st["side_entries"]]
    assert any(used) and not all(used), st
    if cx:
        assert st["records"][0] > 0 and st["records"][1] > 0, st  # steady passes: records only
        compact = (0, 1, 2, 4, 5, 6, 8)  # ticks on 2, 5, 8; dense on 3, 7
        assert all(st["records"][k] > 0 for k in compact) and not any(st["side_entries"][k] for k in compact), st
        assert any(st["side_entries"][k] > 0 for k in (3, 7)), st  # cold fields, dense form


def test_cx_pack_unpack(gpu):
    """gr_space_cx_pack/_unpack on the device equal the host codec: every mailbox
    of a space (uniform compact Replicates and accepts as records, heartbeats and
    multi-entry Replicates as full entries, a LogIndex whose high bits differ from
    its wave's as a full entry) lands in the target space; with small capacities
    the records overflow into full entries and those past the full capacity
    arrive as lost (MB_COLD_LOST)."""
    import torch
    from dragonboat_amd import abi
    from dragonboat_amd.engine import Engine, decode_space, cx_caps_array
    eng = Engine(64, 3)
    lib = eng.lib
    n_chunks, positions, depth = 3, 1000, 3
    rng = np.random.default_rng(9)
    msgs, pos = [], []
    for c in range(n_chunks):
        for q in range(positions):
            if rng.random() < 0.3:
                continue
            kind = rng.integers(0, 4)
            base = (c << 20) + q
            for k in range(1 if kind != 1 else 2):
                m = np.zeros(1, abi.MESSAGE)[0]
                m["term"] = 7
                if kind in (0, 1):  # compact Replicate(s) at one LogIndex (a shared pair for kind 1)
                    m["type"] = abi.REPLICATE
                    m["log_index"] = (2**32 if q % 97 else 2**33) + base
                    m["log_term"] = 7
                    m["commit"] = m["log_index"] - 3 + k
                    m["n_entries"] = k
                    m["n_runs"] = k
                    m["run_term"][0] = 7 if k else 0
                elif kind == 2:
                    m["type"] = abi.HEARTBEAT
                    m["commit"] = base
                    m["hint"] = base + 5
                else:
                    m["type"] = abi.REPLICATE_RESP
                    m["log_index"] = 2**32 + base
                msgs.append(m)
                pos.append(c * X_pad(positions) + q)
    msgs = np.array(msgs, abi.MESSAGE)
    pos = np.array(pos, np.uint32)
    nb = eng.space_bytes(n_chunks, positions, depth)
    src = np.zeros(nb, np.uint8)
    assert lib.gr_space_encode(src.ctypes.data, n_chunks, positions, depth, msgs.ctypes.data, len(msgs),
                               pos.ctypes.data) == 0
    want = decode_space(src.copy(), n_chunks, positions, depth, lost_ok=True)
    for cap, scap in [(positions, positions), (200, 100)]:
        cb = eng.cx_bytes(n_chunks, positions, depth, cap, scap)
        h_cx = np.zeros(cb, np.uint8)
        h_dst = np.full(nb, 0x5A, np.uint8)
        caps = cx_caps_array(cap, n_chunks)
        assert lib.gr_space_cx_pack_host(src.ctypes.data, n_chunks, positions, depth, h_cx.ctypes.data,
                                         caps.ctypes.data, scap) == 0
        assert lib.gr_space_cx_unpack_host(h_dst.ctypes.data, n_chunks, positions, depth, h_cx.ctypes.data,
                                           caps.ctypes.data, scap) == 0
        d_src = torch.from_numpy(src).cuda()
        d_cx = torch.zeros(cb, dtype=torch.uint8, device="cuda")
        d_dst = torch.full((nb,), 0x5A, dtype=torch.uint8, device="cuda")
        eng.cx_pack(d_src.data_ptr(), n_chunks, positions, depth, d_cx.data_ptr(), cap, scap)
        eng.cx_unpack(d_dst.data_ptr(), n_chunks, positions, depth, d_cx.data_ptr(), cap, scap)
        torch.cuda.synchronize()
        got_h = decode_space(h_dst, n_chunks, positions, depth, lost_ok=True)
        got_d = decode_space(d_dst.cpu().numpy(), n_chunks, positions, depth, lost_ok=True)
        key = lambda a: np.sort(a, order=["peer", "type", "log_index", "commit", "hint"])
        lost = got_d["reject"] == 0xFF
        if cap >= positions:
            assert np.array_equal(key(got_h), key(got_d))
            assert not lost.any()
            assert np.array_equal(key(got_d), key(want))
        else:
            # which mailboxes fit depends on the packer's order (the device's
            # waves take record slots in atomic order, the host in position
            # order), how many do not: every mailbox arrives whole or as lost
            lost_h = got_h["reject"] == 0xFF
            assert lost.any()
            assert len(np.unique(got_d["peer"][~lost])) == len(np.unique(got_h["peer"][~lost_h]))
            ok = np.isin(want["peer"], got_d["peer"][~lost])
            assert np.array_equal(key(got_d[~lost]), key(want[ok]))
            assert set(np.unique(want["peer"])) == set(np.unique(got_d["peer"]))
    eng.close()


def X_pad(positions):
    from dragonboat_amd.exchange import pad_positions
    return pad_positions(positions)


def test_side_buffer_pack_unpack(gpu):
    """gr_space_side_pack/_unpack on the device equal the host codec: the cold
    fields of every non-uniform mailbox land in the target space, and the ones
    beyond the capacity are marked MB_COLD_LOST."""
    import torch
    from dragonboat_amd import abi
    from dragonboat_amd.engine import load_library, decode_space
    lib = load_library()
    n_chunks, positions, depth = 2, 4096, 3
    nb = int(lib.gr_space_bytes(n_chunks, positions, depth))
    rng = np.random.default_rng(4)
    msgs, pos = [], []
    pc = (positions + 255) // 256 * 256
    for c in range(n_chunks):
        for q in rng.choice(positions, 900, replace=False):
            for k in range(int(rng.integers(1, depth + 1))):
                m = np.zeros(1, abi.MESSAGE)[0]
                m["term"] = 3
                m["type"] = abi.HEARTBEAT if rng.random() < 0.6 else abi.REPLICATE
                m["log_index"] = int(rng.integers(1, 2**40))
                m["log_term"] = 3
                m["commit"] = m["log_index"]
                m["hint"] = int(rng.integers(0, 2**63))
                m["hint_high"] = q
                msgs.append(m)
                pos.append(c * pc + int(q))
    msgs = np.array(msgs, abi.MESSAGE)
    order = np.argsort(np.array(pos), kind="stable")
    msgs, pos = msgs[order], np.array(pos, np.uint32)[order]
    src = np.zeros(nb, np.uint8)
    assert lib.gr_space_encode(src.ctypes.data, n_chunks, positions, depth, msgs.ctypes.data, len(msgs),
                               pos.ctypes.data) == 0
    for cap in (4096, 100):
        sb = int(lib.gr_space_side_bytes(n_chunks, depth, cap))
        d_src = torch.from_numpy(src.copy()).cuda()
        d_side = torch.zeros(sb, dtype=torch.uint8, device="cuda")
        assert lib.gr_space_side_pack(d_src.data_ptr(), n_chunks, positions, depth, d_side.data_ptr(), cap, None) == 0
        # the receiver: the hot region only, then the side buffers
        hot = int(lib.gr_space_hot_chunk_bytes(positions, depth)) * n_chunks
        d_dst = torch.zeros(nb, dtype=torch.uint8, device="cuda")
        d_dst[:hot] = d_src[:hot]
        assert lib.gr_space_side_unpack(d_dst.data_ptr(), n_chunks, positions, depth, d_side.data_ptr(), cap,
                                        None) == 0
        torch.cuda.synchronize()
        # host codec on the same input
        h_src, h_side = src.copy(), np.zeros(sb, np.uint8)
        assert lib.gr_space_side_pack_host(h_src.ctypes.data, n_chunks, positions, depth, h_side.ctypes.data,
                                           cap) == 0
        h_dst = np.zeros(nb, np.uint8)
        h_dst[:hot] = h_src[:hot]
        assert lib.gr_space_side_unpack_host(h_dst.ctypes.data, n_chunks, positions, depth, h_side.ctypes.data,
                                             cap) == 0
        got = decode_space(d_dst.cpu().numpy(), n_chunks, positions, depth, lost_ok=True)
        want = decode_space(h_dst, n_chunks, positions, depth, lost_ok=True)
        full = decode_space(src, n_chunks, positions, depth)
        lost_d, lost_h = got["reject"] == 0xFF, want["reject"] == 0xFF
        if cap == 4096:
            assert not lost_d.any() and not lost_h.any()
            assert np.array_equal(got, full) and np.array_equal(want, full)
        else:
            # the same number of mailboxes lost either way (which ones depends on
            # the order of the device's appends); every delivered one exact
            n_lost = lambda r: len(set(int(x) for x in r["peer"][r["reject"] == 0xFF]))  # mailboxes
            assert n_lost(got) == n_lost(want) > 0
            keep = ~lost_d
            idx = {(int(m["peer"]), int(m["slot"])): m for m in full}
            assert all(np.array_equal(np.array([idx[(int(m["peer"]), int(m["slot"]))]]), np.array([m]))
                       for m in got[keep])


def test_bench_runs(gpu):
    """bench.py's contract on a small population (JSON line with roofline)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--groups", "20000", "--steps", "5",
                        "--warmup", "3", "--cpu-baseline", "off"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["value"] > 0 and line["escalations"] == 0
    assert line["roofline"]["achieved"] > 0


def test_gpu_config3_read_index_quiesced(gpu):
    """BASELINE config 3 shape on the GPU (R=5, slots=5 kernels)."""
    R, G = 5, 1000
    peers, active = P.config3(G, R)
    topo = P.Topology(G, R)
    rng = np.random.default_rng(33)
    st = SIM.simulate(SIM.GpuBackend, peers, topo, 8, lambda k: P.config3_locals(G, R, active, k),
                      slots=R, drop_fn=lambda k, m: P.drop_acks(m, 0.1, rng))
    assert st["ready"] > 0


def test_full_size_properties(gpu):
    """The bench population at full size (1M groups x 3, device-resident path, 8
    passes): no escalation or hand-over, every group's commit and log advanced by
    the same amounts, and a 64-group sample equal field by field to the oracle run
    on the same records and inputs."""
    import torch
    from dragonboat_amd.engine import Engine
    from dragonboat_amd.exchange import Exchange
    from oracle.pyoracle import OraclePopulation
    import parity
    from dragonboat_amd import abi
    G, R, S, K = 1_000_000, 3, 3, 8
    ex = Exchange(G, R, S, 1, 0, "local")
    n = ex.n_peers
    eng = Engine(n, S)
    eng.load(ex.peers)
    eng.bind_routes(ex.in_pos, ex.out_pos)
    eng.set_locals(P.propose_locals(n, ex.leader_slots, pass_index=0))
    spaces = ex.allocate(eng, torch.device("cuda", 0))
    stream = torch.cuda.current_stream()
    for k in range(K):
        ex.step(eng, spaces, k, stream)
    torch.cuda.synchronize()
    st = eng.stats()
    assert st["escalations"] == 0
    final = eng.sync(n)
    eng.close()
    hi0 = ex.peers["last_index"].astype(np.int64)
    dc = final["committed"].astype(np.int64) - hi0
    dl = final["last_index"].astype(np.int64) - hi0
    for r in range(R):
        blk = slice(r * G, (r + 1) * G)
        assert np.all(dc[blk] == dc[r * G]), f"replica {r}: committed deltas differ"
        assert np.all(dl[blk] == dl[r * G]), f"replica {r}: lastIndex deltas differ"
    # leader: K proposals, commit two passes behind; followers one pass behind the leader
    assert (dc[0], dl[0]) == (K - 2, K) and (dc[G], dl[G]) == (K - 3, K - 1)
    # oracle on a 64-group sample of the same records (replica-major re-indexed)
    g0 = 64
    idx = np.concatenate([np.arange(r * G, r * G + g0) for r in range(R)])
    sample = ex.peers[idx].copy()
    pop = OraclePopulation(sample, S)
    topo = P.Topology(g0, R)
    msgs = np.zeros(0, abi.MESSAGE)
    for k in range(K):
        o = pop.step(msgs, P.propose_locals(R * g0, np.arange(g0), pass_index=0))
        msgs = topo.route_messages(o["msgs"])
    bad = parity.compare_states(final[idx], pop.export(), S)
    assert not bad, bad[:3]


def test_load_sync_round_trip(gpu):
    """gr_load_groups/gr_sync_groups_to_host and the slot-list variants
    (gr_load_peers/gr_sync_peers_to_host) transpose records <-> state rows on the
    device: every field comes back; bad input is refused before any row changes."""
    from dragonboat_amd import abi
    from dragonboat_amd.engine import Engine, GpuRaftError
    import parity
    G, R = 3000, 5
    peers, _ = P.config3(G, R)
    topo = P.Topology(G, R)
    P.inject_leader_change(peers, topo, 0.2, np.random.default_rng(1))
    n = len(peers)
    eng = Engine(n, R)
    eng.load(peers)
    assert not parity.compare_states(eng.sync(n), peers, R)
    # scattered slots, shuffled order
    rng = np.random.default_rng(2)
    slots = rng.permutation(n)[: n // 3].astype(np.uint32)
    fresh = P.make_groups(G, R, seed=9)[: len(slots)]
    eng.load_peers(slots, fresh)
    got = eng.sync_peers(slots)
    assert not parity.compare_states(got, fresh, R)
    whole = eng.sync(n)
    keep = np.setdiff1d(np.arange(n), slots)
    assert not parity.compare_states(whole[keep], peers[keep], R)
    before = eng.sync(n)
    for bad_slots in (np.array([1, 2, 1], np.uint32), np.array([0, n], np.uint32)):
        with pytest.raises(GpuRaftError):
            eng.load_peers(bad_slots, fresh[: len(bad_slots)])
    broken = fresh[:2].copy()
    broken["n_runs"][1] = abi.GR_K + 1
    with pytest.raises(GpuRaftError):
        eng.load_peers(np.array([5, 6], np.uint32), broken)
    assert not parity.compare_states(eng.sync(n), before, R)  # nothing written
    eng.close()


def _interleave(msgs, rng):
    """A random arrival order that keeps each mailbox's (peer, slot) own order."""
    n = len(msgs)
    perm = rng.permutation(n)
    key = msgs["peer"].astype(np.int64) * 256 + msgs["slot"]
    order = np.empty(n, np.int64)
    for k in np.unique(key):
        idx = np.nonzero(key == k)[0]          # original order within the mailbox
        order[np.sort(perm[idx])] = idx        # the shuffled slots this mailbox got
    return msgs[order]


def test_gr_step_boundary_order_and_edges(gpu):
    """gr_step's device boundary (gr_io.h): lanes, mailbox order and records do not
    depend on how mailboxes interleave in the inbox; a mailbox given more than GR_C
    messages escalates CAPACITY at the first that did not travel; the last local
    record of a peer wins; a bad record fails the call before any state changes."""
    from dragonboat_amd import abi
    from dragonboat_amd.engine import Engine, GpuRaftError
    import parity
    G, R = 400, 3
    peers = P.make_groups(G, R, seed=4)
    topo = P.Topology(G, R)
    P.inject_leader_change(peers, topo, 0.3, np.random.default_rng(4))
    a, b = Engine(R * G, R), Engine(R * G, R)
    a.load(peers)
    b.load(peers)
    rng = np.random.default_rng(5)
    msgs = np.zeros(0, abi.MESSAGE)
    for k in range(6):
        loc = P.propose_locals(R * G, P.current_leaders(a.sync(R * G), topo), pass_index=k)
        oa, ra = a.step(msgs, loc)
        ob, rb = b.step(_interleave(msgs, rng), loc[rng.permutation(len(loc))])
        assert np.array_equal(oa, ob) and np.array_equal(ra, rb)
        assert not parity.compare_states(a.sync(R * G), b.sync(R * G), R)
        msgs = topo.route_messages(oa)
    # more than GR_C messages in one mailbox
    st = a.sync(R * G)
    f = int(np.nonzero(st["state"] == abi.FOLLOWER)[0][0])
    hb = np.zeros(abi.GR_C + 2, abi.MESSAGE)
    hb["peer"], hb["type"], hb["term"] = f, abi.HEARTBEAT, st["term"][f]
    hb["slot"] = next(j for j in range(R) if j != st["self_slot"][f])
    _, res = a.step(hb, None)
    r = res[res["peer"] == f][0]
    assert abi.ESC_NAMES[r["escalation"]] == "capacity" and r["esc_item"] == abi.GR_C
    # the last local record of a peer wins
    loc = np.zeros(2, abi.LOCAL)
    loc["peer"] = f
    loc["ticks"] = [3, 1]
    before = a.sync(R * G)[f]["election_tick"]
    a.step(None, loc)
    assert a.sync(R * G)[f]["election_tick"] == before + 1
    # bad records: nothing runs
    snap = a.sync(R * G)
    bad = hb[:2].copy()
    bad["slot"][1] = R  # out of range
    with pytest.raises(GpuRaftError):
        a.step(bad, None)
    assert not parity.compare_states(a.sync(R * G), snap, R)
    a.close()
    b.close()


# ---- BASELINE.json configs 2, 3 and 5 at their full sizes, bit-exact against the
# oracle after every pass (gr_step path; SIM.simulate compares state, messages and
# results of every peer).

def test_baseline_config2_full_size(gpu):
    """configs[1]: 10k groups x 3 replicas, uniform proposals."""
    st = _sim(10_000, 8, seed=2)
    assert st["escalations"] == 0 and st["commits"] >= 10_000 * 6


def test_baseline_config3_full_size(gpu):
    """configs[2]: 100k groups x 5, 90% quiesced, ReadIndex on the active 10%,
    acks dropped with p = 0.1, ticks, CheckQuorum on half."""
    R, G = 5, 100_000
    peers, active = P.config3(G, R)
    topo = P.Topology(G, R)
    rng = np.random.default_rng(3)
    st = SIM.simulate(SIM.GpuBackend, peers, topo, 4, lambda k: P.config3_locals(G, R, active, k),
                      slots=R, drop_fn=lambda k, m: P.drop_acks(m, 0.1, rng))
    assert st["ready"] > 0


def test_baseline_config5_full_size(gpu):
    """configs[4]: 100k groups x 3 with leader changes injected at p = 0.1 per pass
    (divergent suffixes, rejects, decreaseTo, truncation, forwarded proposals)."""
    G, R = 100_000, 3
    topo = P.Topology(G, R)
    st = _sim(G, 6, seed=5, inject_p=0.1,
              locals_fn=lambda k, cur: P.propose_locals(R * G, P.current_leaders(cur, topo), pass_index=k))
    assert st["commits"] > 0 and st["forwarded"] > 0


def test_baseline_config4_full_size_one_gpu(gpu):
    """configs[3] at N=1: 1M groups x 3 replicas, every peer bit-exact against the
    oracle after each of 3 passes (gr_step path; leaders commit on the third)."""
    st = _sim(1_000_000, 3, seed=4)
    assert st["escalations"] == 0 and st["commits"] > 0


@pytest.mark.gpu
def test_notify_applied_gates_elections(built, gpu):
    """gr_notify_applied = Peer.NotifyRaftLastApplied (peer.go:282) before a pass.
    Followers whose election timeout fires this pass start an election only when
    committed <= applied (handleNodeElection, raft.go:1055-1079): behind applied
    they skip it; after the notify they escalate GR_ESC_ELECTION. Same as the
    oracle given the same applied indexes; other groups untouched."""
    from dragonboat_amd import abi, populations as P
    from dragonboat_amd.engine import Engine
    from oracle.pyoracle import OraclePopulation
    import parity

    G, R, S = 512, 3, 3
    peers = P.make_groups(G, R, seed=17)
    fol = np.nonzero(peers["state"] == abi.FOLLOWER)[0]
    peers["election_tick"][fol] = peers["randomized_election_timeout"][fol] - 1
    peers["applied"][fol] = peers["committed"][fol] - 1
    eng = Engine(R * G, S)
    eng.load(peers)
    slots = fol[::2].astype(np.uint32)
    new_applied = peers["committed"][slots]
    eng.notify_applied(slots, new_applied)
    dev0 = eng.sync(R * G)
    assert (dev0["applied"][slots] == new_applied).all()
    rest = np.setdiff1d(np.arange(R * G), slots)
    assert (dev0["applied"][rest] == peers["applied"][rest]).all()

    want = peers.copy()
    want["applied"][slots] = new_applied
    pop = OraclePopulation(want, S)
    loc = P.propose_locals(R * G, [], ticks=1)
    msgs = np.zeros(0, abi.MESSAGE)
    out, res = eng.step(msgs, loc)
    lim = parity.limits_from(res, R * G)
    o = pop.step(msgs, loc, lim)
    bad = parity.compare_states(eng.sync(R * G), o["mid"], S)
    bad += parity.compare_msgs(out, parity.prefix_msgs(o, lim))
    bad += parity.compare_results(res, o["results"])
    assert bad == [], bad[:3]
    esc = {int(r["peer"]) for r in res if r["escalation"] == 4}  # GR_ESC_ELECTION
    assert esc == set(int(x) for x in slots)
    # refused: a slot out of range or listed twice writes nothing
    with pytest.raises(Exception):
        eng.notify_applied(np.array([0, 0], np.uint32), np.array([1, 2], np.uint64))
    with pytest.raises(Exception):
        eng.notify_applied(np.array([R * G], np.uint32), np.array([1], np.uint64))
    eng.close()


@pytest.mark.gpu
def test_compact_log_moves_first_index(built, gpu):
    """gr_compact_log = LogReader.Compact (logreader.go:251-269) mirrored into
    entryLog.firstIndex. A leader whose lagging follower needs entries below the
    new firstIndex takes the snapshot path (makeReplicateMessage, raft.go:474-498)
    exactly as the oracle with the same firstIndex; uncompacted groups replicate.
    Refusals follow Compact: below firstIndex-1 -> ErrCompacted, past lastIndex ->
    ErrUnavailable, nothing written for those slots."""
    from dragonboat_amd import abi, populations as P
    from dragonboat_amd.engine import Engine
    from oracle.pyoracle import OraclePopulation
    import parity

    G, R, S = 256, 3, 3
    peers = P.make_groups(G, R, seed=23)
    leaders = np.arange(G)  # replica-major: slot g is group g's leader
    hi = peers["last_index"][leaders]
    rem = peers["remotes"]  # field views first: fancy indexing would copy
    rem["match"][leaders, 1] = hi - np.uint64(10)
    rem["next"][leaders, 1] = hi - np.uint64(9)
    eng = Engine(R * G, S)
    eng.load(peers)
    comp = leaders[::2].astype(np.uint32)
    new_lo = peers["last_index"][comp] - np.uint64(5)
    rc, st = eng.compact_log(comp, new_lo)
    assert rc == 0 and (st == 0).all()
    dev0 = eng.sync(R * G)
    assert (dev0["first_index_m1"][comp] == new_lo).all()

    # LogReader.Compact leaves entryLog.applied and the in-memory marks alone: the
    # oracle starts from the loaded marks, then the compacted firstIndex
    want = parity.normalize_marks(peers)
    want["first_index_m1"][comp] = new_lo
    pop = OraclePopulation(want, S)
    loc = P.propose_locals(R * G, leaders, pass_index=0)
    msgs = np.zeros(0, abi.MESSAGE)
    out, res = eng.step(msgs, loc)
    lim = parity.limits_from(res, R * G)
    # The oracle runs the host suffix too: in the reference the escalated item
    # reaches makeInstallSnapshotMessage, whose log has no snapshot here (a Go
    # panic, "got an empty snapshot"); the device prefix is compared.
    o = pop.step(msgs, loc, lim, allow_error=True)
    assert o["error"] == "" or "empty snapshot" in o["error"], o["error"]
    bad = parity.compare_states(eng.sync(R * G), o["mid"], S)
    bad += parity.compare_msgs(out, parity.prefix_msgs(o, lim))
    bad += parity.compare_results(res, o["results"])
    assert bad == [], bad[:3]
    snap = {int(r["peer"]) for r in res if r["escalation"] == 7}  # GR_ESC_SNAPSHOT
    assert snap == set(int(x) for x in comp)

    # Compact's refusals: index below firstIndex-1, index past the persisted lastIndex
    dev1 = eng.sync(R * G)
    probe = np.array([G + 1, G + 2, G + 3], np.uint32)
    idx = np.array([dev1["first_index_m1"][G + 1] - 1, dev1["last_index"][G + 2] + 1,
                    dev1["first_index_m1"][G + 3] + 1], np.uint64)
    rc, st = eng.compact_log(probe, idx)
    assert rc == -6 and list(st) == [1, 2, 0]
    dev2 = eng.sync(R * G)
    assert dev2["first_index_m1"][G + 1] == dev1["first_index_m1"][G + 1]
    assert dev2["first_index_m1"][G + 2] == dev1["first_index_m1"][G + 2]
    assert dev2["first_index_m1"][G + 3] == idx[2]
    # past the persisted end but inside the log (the pass's unsaved append):
    # LogReader.Compact refuses it (its lastIndex is what LogDB holds)
    unsaved = [int(x) for x in np.nonzero(dev2["saved_to"] < dev2["last_index"])[0] if x not in probe]
    assert unsaved, "the pass appended nothing unsaved"  # the proposing leaders did
    p4 = unsaved[0]
    rc, st = eng.compact_log(np.array([p4], np.uint32), np.array([dev2["last_index"][p4]], np.uint64))
    assert rc == -6 and list(st) == [2]
    rc, st = eng.compact_log(np.array([p4], np.uint32), np.array([dev2["saved_to"][p4]], np.uint64))
    assert rc == 0 and list(st) == [0]
    eng.close()


@pytest.mark.parametrize("banks,exchange,codec", [(1, False, "cx"), (1, True, "cx"), (2, True, "cx"),
                                                  (2, True, "dense")])
def test_pipeline_spread_banks(gpu, banks, exchange, codec):
    """The banked spread pipeline (dragonboat_amd.exchange.Pipeline: one engine
    and HIP stream per bank) at N = 1 equals an oracle run of every bank's groups
    after every pass: with the one-rank ping-pong (exchange=False, what bench.py
    runs at N = 1) and with the N > 1 exchange code kept (exchange=True: device
    copy of the hot region, side-buffer pack/unpack)."""
    import torch
    from dragonboat_amd import abi
    from dragonboat_amd.engine import Engine
    from dragonboat_amd.exchange import Pipeline
    from oracle.pyoracle import OraclePopulation
    import parity
    G, R, K = 900, 3, 5
    pipe = Pipeline(G, R, R, 1, 0, "spread", banks=banks, exchange=exchange, codec=codec)
    pipe.setup(Engine, torch.device("cuda", 0), 0)
    pops = [OraclePopulation(ex.peers, R) for ex in pipe.ex]
    msgs = [np.zeros(0, abi.MESSAGE) for _ in pipe.ex]
    try:
        for k in range(K):
            pipe.step(k)
            pipe.synchronize()
            for b, ex in enumerate(pipe.ex):
                loc = P.propose_locals(ex.n_peers, ex.leader_slots, pass_index=0)
                o = pops[b].step(msgs[b], loc)
                msgs[b] = P.Topology(ex.G, R).route_messages(o["msgs"])
                bad = parity.compare_states(pipe.engines[b].sync(ex.n_peers), o["mid"], R)
                assert not bad, (k, b, bad[:2])
        assert sum(e.stats()["leader_commits"] for e in pipe.engines) > 0
    finally:
        pipe.close()
