"""Route tables of the device exchange (dragonboat_amd/exchange.py) and the
multi-rank all_to_all over gloo (CPU): every sender mailbox lands exactly in
the receiver's mailbox for the same (group, sender replica)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dragonboat_amd import exchange as X
from dragonboat_amd import populations as P


def _owner(rank, r, N):
    return (rank - r) % N  # home of the group whose replica r sits on `rank`


@pytest.mark.parametrize("N", [1, 2, 3, 4, 5, 8])
def test_spread_routes_bijection(N):
    G, R, S = 37, 3, 3
    tables = [X.spread_routes(G, R, S, N, a) for a in range(N)]
    ranks = [X.spread_peer_ranks(R, N, a) for a in range(N)]
    positions = tables[0][2]
    pc = X.pad_positions(positions)
    # sender side: (rank a, chunk d, local pos) -> (home, g, r, j)
    sent = {}
    for a in range(N):
        _, out_pos, _ = tables[a]
        for j in range(S):
            for p in range(R * G):
                v = int(out_pos[j, p])
                if v == X.NOPOS:
                    continue
                r, g = divmod(p, G)
                c, loc = divmod(v, pc)
                d = ranks[a][0][c]  # chunk slot -> destination rank
                assert loc < positions
                key = (a, d, loc)
                assert key not in sent
                sent[key] = (_owner(a, r, N), g, r, j)
    recv = {}
    for d in range(N):
        in_pos, _, _ = tables[d]
        for r in range(S):
            for p in range(R * G):
                v = int(in_pos[r, p])
                if v == X.NOPOS:
                    continue
                j, g = divmod(p, G)
                c, loc = divmod(v, pc)
                a = ranks[d][1][c]  # chunk slot -> source rank
                recv[(a, d, loc)] = (_owner(d, j, N), g, r, j)
    assert sent == recv
    assert len(sent) == N * G * R * (R - 1)


@pytest.mark.parametrize("N,want", [(1, 1), (2, 2), (3, 2), (4, 3), (5, 4), (8, 4), (16, 4)])
def test_spread_chunks_only_for_reached_ranks(N, want):
    """At R = 3 a rank exchanges with the ranks at offsets +-1, +-2 only."""
    for a in range(N):
        d, s = X.spread_peer_ranks(3, N, a)
        assert len(d) == len(s) == want
        assert d == sorted(d) and s == sorted(s)


def test_local_routes_match_topology():
    G, R = 50, 3
    ex = X.Exchange(G, R, R, 1, 0, "local")
    inv = {}
    for j in range(R):
        for p in range(R * G):
            v = int(ex.in_pos[j, p])
            if v != X.NOPOS:
                inv[v] = (p, j)
    topo = P.Topology(G, R)
    for j in range(R):
        for p in range(R * G):
            v = int(ex.out_pos[j, p])
            if v == X.NOPOS:
                assert p // G == j
                continue
            dp, ds = topo.dest(p, j)
            assert inv[v] == (int(dp), int(ds))


def test_spread_peers_agree_across_ranks():
    """Every replica of a group, wherever placed, starts from the same group state."""
    G, R, N = 16, 3, 4
    recs = [X.spread_peers(G, R, N, a, seed=5) for a in range(N)]
    for h in range(N):
        reps = [recs[(h + r) % N][r * G:(r + 1) * G] for r in range(R)]
        for r in range(1, R):
            for f in ("term", "last_index", "committed"):
                assert np.array_equal(reps[0][f], reps[r][f])
            assert np.all(reps[r]["node_id"] == r + 1)


def _worker(rank, world, port, G, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R = S = 3
    in_pos, out_pos, positions = X.spread_routes(G, R, S, world, rank)
    dests, srcs = X.spread_peer_ranks(R, world, rank)
    pc = X.pad_positions(positions)
    # each sender writes a tag (rank, replica, group, slot) into its mailboxes
    out = torch.zeros(len(dests) * pc, dtype=torch.int64)
    for j in range(S):
        for p in range(R * G):
            v = int(out_pos[j, p])
            if v != X.NOPOS:
                r, g = divmod(p, G)
                out[v] = 1 + ((rank * 8 + r) * 1000 + g) * 8 + j
    inp = torch.zeros(len(srcs) * pc, dtype=torch.int64)
    # the split sizes Exchange.step passes (in elements here, bytes there)
    dist.all_to_all_single(inp, out, output_split_sizes=[pc if a in srcs else 0 for a in range(world)],
                           input_split_sizes=[pc if d in dests else 0 for d in range(world)])
    errs = 0
    for r in range(S):
        for p in range(R * G):
            v = int(in_pos[r, p])
            if v == X.NOPOS:
                continue
            j, g = divmod(p, G)
            src = (rank - j + r) % world
            want = 1 + ((src * 8 + r) * 1000 + g) * 8 + j
            errs += int(inp[v]) != want
    q.put((rank, errs))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 5])
def test_gloo_all_to_all_delivery(world):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 29, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(e == 0 for _, e in res), res


def _heavy_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pipe = X.Pipeline(128, 3, 3, world, rank, "spread", verify_heavy=True)
    out = []
    for heavy in (False, True, rank == 0):  # agree, agree, disagree
        try:
            pipe._check_heavy(heavy)
            out.append("ok")
        except RuntimeError:
            out.append("refused")
    q.put((rank, out))
    dist.destroy_process_group()


def test_heavy_flag_checked_across_ranks():
    """ranks passing different `heavy` to Pipeline.step would pair
    all-to-all buffers of different sizes; verify_heavy refuses the pass on
    every rank before anything moves."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_heavy_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(o == ["ok", "ok", "refused"] for _, o in res), res


@pytest.mark.parametrize("placement,N,rank", [("local", 1, 0), ("spread", 1, 0), ("spread", 2, 1),
                                              ("spread", 8, 5)])
def test_routes_are_affine(built, placement, N, rank):
    """gr_bind_routes turns the bench topologies into RT_AFFINE routes:
    position = base[dir][replica][slot] + group, reproducing the tables exactly."""
    from oracle.pyoracle import hostlane_affine_routes
    G, R, S = 96, 3, 3
    if placement == "local":
        in_pos, out_pos = P.Topology(G, R).loopback_routes(S)
    else:
        in_pos, out_pos, _ = X.spread_routes(G, R, S, N, rank)
    got = hostlane_affine_routes(in_pos, out_pos, S)
    assert got is not None
    base, g, mode = got
    assert g == G
    assert mode == ("loopback" if placement == "local" else "affine")
    for d, t in enumerate((in_pos, out_pos)):
        for j in range(S):
            for r in range(R):
                b = int(base[d, r, j])
                want = t[j, r * G:(r + 1) * G]
                if b == 0xFFFFFFFF:
                    assert np.all(want == 0xFFFFFFFF)
                else:
                    assert np.array_equal(want, b + np.arange(G, dtype=np.uint32))


def test_routes_not_affine_fall_back(built):
    """A table that is not replica-major affine keeps RT_TABLE."""
    from oracle.pyoracle import hostlane_affine_routes
    G, R, S = 64, 3, 3
    in_pos, out_pos = P.Topology(G, R).loopback_routes(S)
    in_pos = in_pos.copy()
    in_pos[1, 5], in_pos[1, 6] = in_pos[1, 6], in_pos[1, 5]
    assert hostlane_affine_routes(in_pos, out_pos, S) is None


class _SideCodec:
    """The C-ABI's space-size and side-buffer functions (host forms: the same
    codec the device kernels run) for engines that step on the CPU."""

    def space_bytes(self, n, positions, depth):
        return int(self.lib.gr_space_bytes(n, positions, depth))

    def chunk_bytes(self, positions, depth):
        return int(self.lib.gr_space_chunk_bytes(positions, depth))

    def hot_chunk_bytes(self, positions, depth):
        return int(self.lib.gr_space_hot_chunk_bytes(positions, depth))

    def hot_tile_bytes(self, depth):
        return int(self.lib.gr_space_hot_tile_bytes(depth))

    def side_bytes(self, n_chunks, depth, cap):
        return int(self.lib.gr_space_side_bytes(n_chunks, depth, cap))

    def side_pack(self, ptr, n_chunks, positions, depth, side_ptr, cap, stream=0):
        assert self.lib.gr_space_side_pack_host(ptr, n_chunks, positions, depth, side_ptr, cap) == 0

    def side_unpack(self, ptr, n_chunks, positions, depth, side_ptr, cap, stream=0):
        assert self.lib.gr_space_side_unpack_host(ptr, n_chunks, positions, depth, side_ptr, cap) == 0

    def cx_bytes(self, n_chunks, positions, depth, caps, scap):
        from dragonboat_amd.engine import cx_caps_array
        c = cx_caps_array(caps, n_chunks)
        return int(self.lib.gr_space_cx_bytes(n_chunks, positions, depth, c.ctypes.data, scap))

    def cx_pack(self, ptr, n_chunks, positions, depth, cx_ptr, caps, scap, stream=0):
        from dragonboat_amd.engine import cx_caps_array
        c = cx_caps_array(caps, n_chunks)
        assert self.lib.gr_space_cx_pack_host(ptr, n_chunks, positions, depth, cx_ptr, c.ctypes.data, scap) == 0

    def cx_unpack(self, ptr, n_chunks, positions, depth, cx_ptr, caps, scap, stream=0):
        from dragonboat_amd.engine import cx_caps_array
        c = cx_caps_array(caps, n_chunks)
        assert self.lib.gr_space_cx_unpack_host(ptr, n_chunks, positions, depth, cx_ptr, c.ctypes.data, scap) == 0


class _MockEngine(_SideCodec):
    """A no-op pass: lets Exchange.step's collectives run over gloo on CPU tensors."""

    def __init__(self):
        from dragonboat_amd.engine import load_library
        self.lib = load_library()

    def step_device(self, *a, **k):
        pass


def _encode_chunks(lib, ex, rank, out):
    """Messages the 'kernel' of `rank` writes into its out space: per destination
    chunk, uniform compact Replicates in some mailboxes and heartbeats (cold
    fields) in others, each message tagged with (rank, destination, position).
    Returns {dest rank: records with peer = position in chunk}."""
    import ctypes
    from dragonboat_amd import abi
    want = {}
    msgs, pos = [], []
    pc = X.pad_positions(ex.positions)
    for c, d in enumerate(ex.dests):
        recs = []
        for q in range(0, ex.positions, 7):
            m = np.zeros(1, abi.MESSAGE)[0]
            m["term"] = 5
            if q % 3:
                m["type"] = abi.REPLICATE
                m["log_index"] = 1000 * rank + 10 * d + q
                m["log_term"] = 5
                m["commit"] = m["log_index"]
            else:
                m["type"] = abi.HEARTBEAT
                m["commit"] = 7 + q
                m["hint"] = (rank << 32) | (d << 16) | q
                m["hint_high"] = q + 1
            msgs.append(m)
            pos.append(c * pc + q)
            r = m.copy()
            r["peer"] = q
            recs.append(r)
        want[d] = recs
    msgs = np.array(msgs, abi.MESSAGE)
    pos = np.array(pos, np.uint32)
    buf = out.numpy()
    assert lib.gr_space_encode(buf.ctypes.data, ex.n_chunks, ex.positions, ex.depth, msgs.ctypes.data, len(msgs),
                               pos.ctypes.data) == 0
    return want


def _step_worker(rank, world, port, side_min, codec, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dragonboat_amd.engine import decode_space

    class _S:
        cuda_stream = 0
    X.SIDE_MIN, X.SIDE_DIV = side_min, 1 << 30
    X.CX_SIDE_MIN, X.CX_SIDE_DIV = side_min, 1 << 30
    G, R = 40, 3
    ex = X.Exchange(G, R, R, world, rank, "spread", codec=codec)
    eng = _MockEngine()
    spaces = ex.allocate(eng, torch.device("cpu"))
    mine = _encode_chunks(eng.lib, ex, rank, spaces[1])
    # every rank's messages for every other rank, as the senders encoded them
    allw = [None] * world
    dist.all_gather_object(allw, {d: [tuple(int(x) for x in (m["peer"], m["type"], m["log_index"], m["commit"],
                                                                m["hint"], m["hint_high"])) for m in v]
                                  for d, v in mine.items()})
    ex.step(eng, spaces, 0, _S())
    got = decode_space(spaces[0].numpy().copy(), ex.n_chunks, ex.positions, ex.depth, lost_ok=True)
    pc = X.pad_positions(ex.positions)
    errs, lost = 0, 0
    for c, a in enumerate(ex.srcs):  # in chunk c came from rank a
        exp = {w[0]: w for w in allw[a][rank]}
        seen = set()
        for m in got:
            if int(m["peer"]) // pc != c:
                continue
            qp = int(m["peer"]) % pc
            if m["reject"] == 0xFF:  # cold fields lost: the count byte says so
                lost += 1
                seen.add(qp)
                continue
            t = (qp, int(m["type"]), int(m["log_index"]), int(m["commit"]), int(m["hint"]), int(m["hint_high"]))
            errs += int(exp.get(qp) != t)
            seen.add(qp)
        errs += len(set(exp) - seen)
    q.put((rank, errs, lost))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,side_min,codec", [(2, 1024, "dense"), (3, 1024, "dense"), (5, 1024, "dense"),
                                                  (3, 2, "dense"), (2, 1024, "cx"), (5, 1024, "cx"), (3, 2, "cx")])
def test_gloo_spread_step_side_buffers(built, world, side_min, codec):
    """Exchange.step over gloo: every mailbox reaches the rank it was written for.
    dense: the hot region whole, the cold fields of the non-uniform mailboxes
    (heartbeats) through the fixed-size side buffers; cx: the compact buffers
    (records for the uniform Replicates, full entries for the heartbeats). With a
    full-entry capacity of 2 the heartbeats beyond it are not lost silently:
    their count bytes carry MB_COLD_LOST (a reading lane escalates CAPACITY)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_step_worker, args=(r, world, port, side_min, codec, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(e == 0 for _, e, _ in res), res
    if side_min >= 1024:
        assert all(lost == 0 for _, _, lost in res), res
    else:
        assert all(lost > 0 for _, _, lost in res), res


class _HostlaneEngine(_SideCodec):
    """A rank's engine for the CPU rehearsal of config 4: the kernels' lane code
    compiled for the host (hl_step) stepping the rank's replicas, reading and
    writing the same mailbox spaces (gr_space_decode/encode) that Exchange.step
    moves between ranks with all_to_all over gloo."""

    def __init__(self, ex):
        from dragonboat_amd.engine import load_library
        self.lib = load_library()
        self.ex = ex
        self.peers = ex.peers.copy()
        self.S = ex.S
        self.k = 0
        self.inv = {}  # mailbox position -> (receiving peer, sender slot)
        for j in range(ex.S):
            for p in np.nonzero(ex.in_pos[j] != X.NOPOS)[0]:
                self.inv[int(ex.in_pos[j, p])] = (int(p), j)

    def step_device(self, in_ptr, out_ptr, in_chunks, in_positions, out_chunks, out_positions, n_peers, stream,
                    depth=3):
        import ctypes
        from dragonboat_amd import abi
        from dragonboat_amd.engine import decode_space
        from oracle.pyoracle import hostlane_step
        ex = self.ex
        nbytes = self.space_bytes(in_chunks, in_positions, depth)
        buf = np.ctypeslib.as_array(ctypes.cast(in_ptr, ctypes.POINTER(ctypes.c_uint8)), (nbytes,))
        got = decode_space(buf.copy(), in_chunks, in_positions, depth)
        msgs = got.copy()
        for m in msgs:
            m["peer"], m["slot"] = self.inv[int(m["peer"])]
        order = np.lexsort((np.arange(len(msgs)), msgs["slot"], msgs["peer"]))
        msgs = msgs[order]
        loc = P.propose_locals(ex.n_peers, ex.leader_slots, pass_index=self.k)
        self.peers, out, res = hostlane_step(self.peers, msgs, loc, self.S)
        assert not np.any(res["escalation"]), res[res["escalation"] != 0][:3]
        ob = np.ctypeslib.as_array(ctypes.cast(out_ptr, ctypes.POINTER(ctypes.c_uint8)), (nbytes,))
        ob[:] = 0
        pos = ex.out_pos[out["slot"].astype(np.int64), out["peer"].astype(np.int64)].astype(np.uint32)
        assert np.all(pos != X.NOPOS)
        out = np.ascontiguousarray(out)
        rc = self.lib.gr_space_encode(ob.ctypes.data, out_chunks, out_positions, depth,
                                      out.ctypes.data if len(out) else None, len(out),
                                      pos.ctypes.data if len(pos) else None)
        assert rc == 0, rc
        self.k += 1

    def cold_used(self, ptr, n_chunks, positions, depth, stream):
        import ctypes
        hb = self.hot_chunk_bytes(positions, depth)
        buf = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), (n_chunks * hb,))
        cnt = X.count_bytes(buf, n_chunks, hb, self.hot_tile_bytes(depth), positions)
        return bool(np.any(((cnt & 7) != 0) & ((cnt & 8) == 0)))


def _raft_worker(rank, world, port, G, passes, codec, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class _S:
        cuda_stream = 0
    R = 3
    ex = X.Exchange(G, R, R, world, rank, "spread", seed=11, codec=codec)
    eng = _HostlaneEngine(ex)
    spaces = ex.allocate(eng, torch.device("cpu"))
    states = []
    for k in range(passes):
        ex.step(eng, spaces, k, _S())
        states.append(eng.peers.copy())
    q.put((rank, states, 0))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,codec", [(2, "dense"), (3, "dense"), (2, "cx"), (3, "cx")])
def test_gloo_spread_raft_matches_oracle(built, world, codec):
    """Config 4 rehearsed on CPU: every rank steps its replicas with the kernels'
    lane code (host build), the Replicate/ReplicateResp mailboxes cross ranks
    through Exchange.step's all_to_all_single (gloo), and after every pass each
    rank's replicas equal a single-process oracle run of the same groups (one
    population per home rank, messages routed inside each group)."""
    import socket
    from dragonboat_amd import abi
    from oracle.pyoracle import OraclePopulation
    import parity
    G, R, passes = 48, 3, 6
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_raft_worker, args=(r, world, port, G, passes, codec, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, states, _cold = q.get(timeout=300)
        res[rank] = states
    for p in procs:
        p.join(timeout=60)
    # the oracle: each home's groups in one process, routed within the group
    topo = P.Topology(G, R)
    orc = {}
    for h in range(world):
        peers = P.make_groups(G, R, seed=int(np.random.SeedSequence(X.group_seed(11, h)).generate_state(1)[0]))
        pop = OraclePopulation(peers, R)
        msgs = np.zeros(0, abi.MESSAGE)
        orc[h] = []
        for k in range(passes):
            o = pop.step(msgs, P.propose_locals(R * G, np.arange(G), pass_index=k))
            orc[h].append(pop.export())
            msgs = topo.route_messages(o["msgs"])
    for rank in range(world):
        for k in range(passes):
            dev = res[rank][k]
            for r in range(R):
                h = (rank - r) % world
                sl = slice(r * G, (r + 1) * G)
                bad = parity.compare_states(dev[sl], orc[h][k][sl], R)
                assert not bad, (rank, k, r, bad[:2])
    assert all(int(res[r][-1]["committed"][:G].min()) > int(res[r][0]["committed"][:G].min()) for r in res)


def test_cx_codec_round_trip(built):
    """The compact exchange's host codec (gr_space_cx_pack_host / _unpack_host,
    the device kernels' logic): a space of uniform compact Replicates and accepts
    (records), heartbeats and multi-entry Replicates (full entries) and empty
    mailboxes unpacks to the same messages; with small capacities the overflow
    is marked lost, never silently dropped; the designed steady-state volume at
    N = 8 and 1M groups per GPU stays under 70 MB per pass."""
    from dragonboat_amd import abi
    from dragonboat_amd.engine import load_library, decode_space
    lib = load_library()
    n_chunks, positions, depth = 2, 700, 3
    rng = np.random.default_rng(3)
    msgs, pos = [], []
    pc = X.pad_positions(positions)
    for c in range(n_chunks):
        for q in range(positions):
            kind = rng.integers(0, 5)
            if kind == 4:
                continue
            for k in range(1 if kind != 1 else 3):
                m = np.zeros(1, abi.MESSAGE)[0]
                m["term"] = 9
                if kind in (0, 1):
                    m["type"] = abi.REPLICATE
                    m["log_index"] = 2**32 + q + 10 * k if q % 50 else 2**34 + q
                    m["log_term"] = 9
                    m["commit"] = m["log_index"] - 1 if q % 13 else m["log_index"] + 2**30
                elif kind == 2:
                    m["type"] = abi.HEARTBEAT
                    m["commit"] = q
                    m["hint"] = q + 1
                else:
                    m["type"] = abi.REPLICATE_RESP
                    m["log_index"] = 2**32 + q
                msgs.append(m)
                pos.append(c * pc + q)
    msgs = np.array(msgs, abi.MESSAGE)
    pos = np.array(pos, np.uint32)
    nb = int(lib.gr_space_bytes(n_chunks, positions, depth))
    src = np.zeros(nb, np.uint8)
    assert lib.gr_space_encode(src.ctypes.data, n_chunks, positions, depth, msgs.ctypes.data, len(msgs),
                               pos.ctypes.data) == 0
    want = decode_space(src.copy(), n_chunks, positions, depth)
    key = lambda a: np.sort(a, order=["peer", "slot", "type", "log_index", "commit", "hint"])
    from dragonboat_amd.engine import cx_caps_array
    for cap, scap, expect_lost in [(pc, pc, False), ([64, 128], 16, True)]:
        caps = cx_caps_array(cap, n_chunks)
        cb = int(lib.gr_space_cx_bytes(n_chunks, positions, depth, caps.ctypes.data, scap))
        cx = np.zeros(cb, np.uint8)
        dst = np.full(nb, 0xA5, np.uint8)  # every count byte is rewritten
        assert lib.gr_space_cx_pack_host(src.ctypes.data, n_chunks, positions, depth, cx.ctypes.data,
                                         caps.ctypes.data, scap) == 0
        assert lib.gr_space_cx_unpack_host(dst.ctypes.data, n_chunks, positions, depth, cx.ctypes.data,
                                           caps.ctypes.data, scap) == 0
        got = decode_space(dst, n_chunks, positions, depth, lost_ok=True)
        lost = got["reject"] == 0xFF
        assert bool(lost.any()) == expect_lost
        ok = np.isin(want["peer"], got["peer"][~lost])
        assert np.array_equal(key(got[~lost]), key(want[ok]))
        assert np.array_equal(np.unique(got["peer"]), np.unique(want["peer"]))  # lost ones still arrive, marked
    # the design volume (exchange.py cx_capacities): N = 8, G = 1M per GPU, R = 3
    _, _, positions8 = X.spread_routes(64, 3, 3, 8, 0)
    pos = positions8 // 64 * 1_000_000
    dests, _ = X.spread_peer_ranks(3, 8, 0)
    tot = 0
    for d in dests:
        cap, scap = X.cx_capacities(pos, X.cx_fill_max(3, 8, d % 8))
        tot += int(lib.gr_space_cx_bytes(1, pos, 3, cx_caps_array([cap], 1).ctypes.data, scap))
    # records for the worst leader placement: 3 chunk-fills of 2M
    # positions x 12 B + wave headers + 1/256 full entries
    assert tot < 90e6, tot


def test_cx_capacity_covers_any_leader_placement():
    """Sized by cx_fill_max, a chunk's record capacity holds the steady state
    whichever replica leads every group (the worst case; mixed leaders fill
    less), at N = 1..8 (leaders moved off replica 0 overflowed)."""
    for N in range(1, 9):
        pairs = X.offset_pairs(3, N)
        per = max(len(v) for v in pairs.values())
        positions = per * 1024
        for o, lst in pairs.items():
            if not lst:
                continue
            cap, _ = X.cx_capacities(positions, X.cx_fill_max(3, N, o))
            for leader in range(3):
                used = sum(1024 for r, j in lst if leader in (r, j))
                assert used <= cap, (N, o, leader, used, cap)


def _tick_space(n_chunks, positions, seed=5):
    """Mailboxes of a tick pass (and near misses): [Replicate, Heartbeat,
    Replicate] from a leader, [accept, HeartbeatResp, accept] from a follower,
    a lone Heartbeat or HeartbeatResp, and variants the pattern records must
    refuse (a context in the heartbeat, accepts out of sequence, a heartbeat
    Commit that differs from the Replicates', a second entry). Returns the
    messages, their positions, and per position whether it must travel as a
    record."""
    from dragonboat_amd import abi
    rng = np.random.default_rng(seed)
    pc = X.pad_positions(positions)
    msgs, pos, want_rec = [], [], {}

    def mk(**f):
        m = np.zeros(1, abi.MESSAGE)[0]
        for k, v in f.items():
            m[k] = v
        return m
    for c in range(n_chunks):
        for q in range(positions):
            kind = int(rng.integers(0, 14))
            T = 5 + (q % 3)
            L = 2**32 + 1000 * q + 7
            C = L - 2
            rep = lambda n, c=C: mk(type=abi.REPLICATE, term=T, log_index=L, log_term=T, commit=c, n_entries=n,
                                    n_runs=n, run_term=[T if n else 0, 0])
            if kind == 0:
                lst, rec = [rep(0), mk(type=abi.HEARTBEAT, term=T, commit=C), rep(1)], True
            elif kind == 1:
                lst, rec = [mk(type=abi.REPLICATE_RESP, term=T, log_index=L), mk(type=abi.HEARTBEAT_RESP, term=T),
                            mk(type=abi.REPLICATE_RESP, term=T, log_index=L + 1)], True
            elif kind == 2:
                lst, rec = [mk(type=abi.HEARTBEAT, term=T, commit=L)], True
            elif kind == 3:
                lst, rec = [mk(type=abi.HEARTBEAT_RESP, term=T)], True
            elif kind == 4:  # a ReadIndex context travels in full
                lst, rec = [rep(0), mk(type=abi.HEARTBEAT, term=T, commit=C, hint=q + 1, hint_high=3)], False
            elif kind == 5:  # accepts out of sequence
                lst, rec = [mk(type=abi.REPLICATE_RESP, term=T, log_index=L), mk(type=abi.HEARTBEAT_RESP, term=T),
                            mk(type=abi.REPLICATE_RESP, term=T, log_index=L + 5)], False
            elif kind == 6:  # the heartbeat's Commit is not the Replicates'
                lst, rec = [rep(0), mk(type=abi.HEARTBEAT, term=T, commit=C - 1)], False
            elif kind == 7:  # two entries
                lst, rec = [mk(type=abi.REPLICATE, term=T, log_index=L, log_term=T, commit=C, n_entries=2, n_runs=1,
                               run_term=[T, 0]), mk(type=abi.HEARTBEAT, term=T, commit=C)], False
            elif kind == 9:  # a commit broadcast and a proposal, unshared
                lst, rec = [rep(0), rep(1)], True
            elif kind == 10:  # two commit advances and a proposal (after a tick pass)
                lst, rec = [rep(0, C - 1), rep(0), rep(1)], True
            elif kind == 11:  # a Commit step of 2
                lst, rec = [rep(0), rep(1, C + 2)], False
            elif kind == 12:  # two accepts, unshared
                lst, rec = [mk(type=abi.REPLICATE_RESP, term=T, log_index=L),
                            mk(type=abi.REPLICATE_RESP, term=T, log_index=L + 1)], True
            elif kind == 13:  # the acks of the staggered commit advances' Replicates
                lst, rec = [mk(type=abi.REPLICATE_RESP, term=T, log_index=L),
                            mk(type=abi.REPLICATE_RESP, term=T, log_index=L),
                            mk(type=abi.REPLICATE_RESP, term=T, log_index=L + 1)], True
            else:
                continue
            for m in lst:
                msgs.append(m)
                pos.append(c * pc + q)
            want_rec[c * pc + q] = rec
    return np.array(msgs, abi.MESSAGE), np.array(pos, np.uint32), want_rec


def test_cx_pattern_records(built):
    """Round 6: a tick pass's mailboxes (a leader's commit broadcast, heartbeat
    and proposal; a follower's acks around its HeartbeatResp; lone heartbeats
    and acks with an empty context), unshared uniform pairs and the staggered
    commit advances after a tick travel as 12-byte records and unpack to the
    very messages sent, every field; near misses go as full entries."""
    from dragonboat_amd.engine import load_library, decode_space, cx_caps_array
    lib = load_library()
    n_chunks, positions, depth = 2, 900, 3
    msgs, pos, want_rec = _tick_space(n_chunks, positions)
    nb = int(lib.gr_space_bytes(n_chunks, positions, depth))
    src = np.zeros(nb, np.uint8)
    assert lib.gr_space_encode(src.ctypes.data, n_chunks, positions, depth, msgs.ctypes.data, len(msgs),
                               pos.ctypes.data) == 0
    want = decode_space(src.copy(), n_chunks, positions, depth)
    pc = X.pad_positions(positions)
    caps = cx_caps_array(pc, n_chunks)
    cb = int(lib.gr_space_cx_bytes(n_chunks, positions, depth, caps.ctypes.data, pc))
    cx = np.zeros(cb, np.uint8)
    dst = np.full(nb, 0xA5, np.uint8)
    assert lib.gr_space_cx_pack_host(src.ctypes.data, n_chunks, positions, depth, cx.ctypes.data,
                                     caps.ctypes.data, pc) == 0
    assert lib.gr_space_cx_unpack_host(dst.ctypes.data, n_chunks, positions, depth, cx.ctypes.data,
                                       caps.ctypes.data, pc) == 0
    got = decode_space(dst, n_chunks, positions, depth)
    key = lambda a: np.sort(a, order=["peer", "slot"])
    assert np.array_equal(key(got), key(want))  # every field of every message
    chunk_bytes = cb // n_chunks
    for c in range(n_chunks):
        n_rec, n_side = X.cx_counts(cx[c * chunk_bytes:(c + 1) * chunk_bytes])
        recs = sum(1 for p, r in want_rec.items() if r and p // pc == c)
        sides = sum(1 for p, r in want_rec.items() if not r and p // pc == c)
        assert (n_rec, n_side) == (recs, sides), (c, n_rec, n_side, recs, sides)
