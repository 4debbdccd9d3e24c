"""Device-resident passes (gr_step_device + mailbox spaces, the bench path)
checked against the oracle after every pass: state, every mailbox of the
written space, and per-peer results."""
import numpy as np

from dragonboat_amd import abi
from dragonboat_amd.engine import Engine, decode_space
from dragonboat_amd.exchange import Exchange
from oracle.pyoracle import OraclePopulation
import parity


def inverse_routes(in_pos):
    """mailbox gpos -> (receiving peer, sender slot) from an in_pos table [S][n]."""
    S, n = in_pos.shape
    inv = {}
    for j in range(S):
        for p in np.nonzero(in_pos[j] != 0xFFFFFFFF)[0]:
            inv[int(in_pos[j, p])] = (int(p), j)
    return inv


def run_device(G, R, passes, placement="local", seed=2, tick_every=0, stats=None, inject_p=0.0, mix=False,
               codec="cx", cx_side=None, heavy_every=0):
    """tick_every > 0: one Tick for every peer on passes k % tick_every == tick_every - 1
    (leader heartbeats and their acks: messages with cold fields).
    inject_p > 0: BASELINE config 5's leader changes (populations.inject_leader_change)
    before every pass after the first, on both sides, proposals on the current leaders.
    mix: peers in a group-major order (peer g*R + r), so every wave holds leaders
    and followers; the routes are then plain tables (local placement only).
    codec: the spread exchange's form ("cx" compact buffers, "dense" hot region +
    side buffers); stats["side_entries"] counts the full entries per pass."""
    import torch
    S = R
    # spread on one rank: keep the exchange (copy + side buffers) under test
    ex = Exchange(G, R, S, 1, 0, placement, seed=seed, exchange=placement == "spread", codec=codec,
                  cx_side=cx_side)
    n = ex.n_peers
    # perm[x] = engine peer of replica-major peer x (identity unless mix)
    perm = np.arange(n)
    if mix:
        assert placement == "local"
        x = np.arange(n)
        perm = (x % G) * R + x // G
        peers = np.empty_like(ex.peers)
        peers[perm] = ex.peers
        ex.peers = peers
        for name in ("in_pos", "out_pos"):
            t = getattr(ex, name)
            t2 = np.empty_like(t)
            t2[:, perm] = t
            setattr(ex, name, t2)
        ex.leader_slots = perm[ex.leader_slots]
    eng = Engine(n, S)
    eng.load(ex.peers)
    eng.bind_routes(ex.in_pos, ex.out_pos)
    from dragonboat_amd import populations as P
    topo = P.Topology(G, R)
    rng = np.random.default_rng(seed + 5)
    def locals_of(k, leaders):
        tk = 1 if tick_every and k % tick_every == tick_every - 1 else 0
        return P.propose_locals(n, leaders, pass_index=0, ticks=tk)
    loc = locals_of(0, ex.leader_slots)
    eng.set_locals(loc)
    spaces = ex.allocate(eng, torch.device("cuda", 0))
    stream = torch.cuda.current_stream()
    pop = OraclePopulation(ex.peers, S)
    inv = inverse_routes(ex.in_pos)
    msgs = np.zeros(0, abi.MESSAGE)  # oracle's view of this pass's inbox
    if stats is not None:
        stats["injected"] = 0
    for k in range(passes):
        if inject_p and k > 0:
            cur = pop.export()
            rm = cur[perm]  # replica-major view for the injector
            ch = P.inject_leader_change(rm, topo, inject_p, rng)
            if len(ch):
                idx = perm[ch]
                pop.reload(idx, rm[ch])
                eng.load_peers(idx.astype(np.uint32), rm[ch])
                if stats is not None:
                    stats["injected"] += len(ch)
            loc = locals_of(k, P.current_leaders(pop.export(), topo))
            eng.set_locals(loc)
        elif tick_every:
            loc = locals_of(k, ex.leader_slots)
            eng.set_locals(loc)
        # heavy_every > 0: passes k % heavy_every == heavy_every - 1 exchange the
        # dense form (Exchange.exchange), the others the compact one
        heavy = bool(heavy_every) and k % heavy_every == heavy_every - 1
        ex.step(eng, spaces, k, stream, heavy=heavy)
        torch.cuda.synchronize()
        if placement == "spread" and stats is not None:  # what the exchange carried
            if ex.last_cx:  # records, full entries (one chunk: headers at offset 0)
                from dragonboat_amd.exchange import cx_counts, CX_HDR
                nrec, nside = cx_counts(ex.cx[1][:CX_HDR].cpu().numpy())
                stats.setdefault("records", []).append(nrec)
                stats.setdefault("side_entries", []).append(nside)
            else:
                sb = len(ex.side[1]) // ex.n_chunks
                hdr = ex.side[1].cpu().numpy().reshape(ex.n_chunks, sb)[:, :4].copy().view(np.uint32)[:, 0]
                stats.setdefault("records", []).append(0)
                stats.setdefault("side_entries", []).append(int(hdr.sum()))
        o = pop.step(msgs, loc)
        res = eng.collect_results(n)
        assert not np.any(res["escalation"]), "unexpected escalation on the device path"
        dev = eng.sync(n)
        bad = parity.compare_states(dev, o["mid"], S)
        assert not bad, f"pass {k}: state {bad[:3]}"
        # the space the next pass reads
        nxt = spaces[(k + 1) % 2] if placement == "local" else spaces[0]
        raw = nxt.cpu().numpy()
        got = decode_space(raw, ex.n_chunks, ex.positions, ex.depth, lost_ok=True)
        # oracle messages -> (receiver, sender slot) records in arrival order
        want = route(o["msgs"], ex, G, R, perm)
        lost = got["reject"] == 0xFF
        if np.any(lost):  # the exchange dropped cold fields: name the pass and what they held
            lp = set(int(x) for x in got["peer"][lost])
            kinds = {}
            for m in want:
                if (int(m["peer"]), int(m["slot"])) in {inv[x] for x in lp}:
                    kinds[int(m["type"])] = kinds.get(int(m["type"]), 0) + 1
            raise AssertionError(f"pass {k} (heavy={heavy}): {len(lp)} mailboxes lost in the exchange, "
                                 f"message types {kinds}, stats {stats}")
        for m in got:
            p, j = inv[int(m["peer"])]
            m["peer"], m["slot"] = p, j
        bad = parity.compare_msgs(got, want)
        assert not bad, f"pass {k}: mailboxes {bad[:3]}"
        bad = parity.compare_results(res, o["results"])
        assert not bad, f"pass {k}: results {bad[:3]}"
        msgs = want
    final = eng.sync(n)
    eng.close()
    return final


def route(out, ex, G, R, perm=None):  # (ex: unused, the layout is replica-major)
    """Outbox records (sender peer, target slot) -> inbox records (receiver, sender slot),
    using the placement's peer layout (replica-major in both placements on one rank,
    engine peer perm[x] for replica-major peer x when given)."""
    nxt = out.copy()
    sender = out["peer"].astype(np.int64)
    if perm is not None:
        inv = np.empty_like(perm)
        inv[perm] = np.arange(len(perm))
        sender = inv[sender]
    r = sender // G
    g = sender % G
    j = out["slot"].astype(np.int64)
    rec = j * G + g
    nxt["peer"] = (perm[rec] if perm is not None else rec).astype(np.uint32)
    nxt["slot"] = r.astype(np.uint8)
    order = np.lexsort((np.arange(len(nxt)), nxt["slot"], nxt["peer"]))
    return nxt[order]


class DeviceLockstep:
    """The device-resident split schedule (gr_step_device over loopback mailbox
    spaces: the steady kernel, the role instances, the tick and general kernels,
    exactly what bench.py and tools/bench_configs.py time) stepped pass by pass
    beside the oracle on identical inputs. After every pass it checks every
    peer's state, every mailbox of the space the next pass reads, every result
    and every escalation against the oracle (the escalation protocol of
    simulate.Lockstep: escalated groups are compared at their prefix and
    reloaded from the oracle's full pass).

    The next pass's inbox is the space the kernels wrote, untouched, unless the
    host has to change it: a group escalated (the space holds only its device
    prefix; the oracle's full outbox is encoded in its place, as the host's
    messages would be) or `drop_fn` drops messages (the network's loss, config
    3's HeartbeatResp drops): then the whole space is re-encoded from the
    oracle's delivered messages (gr_space_encode) and uploaded."""

    def __init__(self, peers, G, R, lib_path=None, threads=16):
        import torch
        from dragonboat_amd import populations as P
        self.G, self.R, self.S = G, R, R
        self.n = R * G
        assert len(peers) == self.n
        self.topo = P.Topology(G, R)
        self.in_pos, self.out_pos = self.topo.loopback_routes(self.S)
        self.positions = self.n * self.S
        self.depth = abi.GR_C
        self.eng = Engine(self.n, self.S, lib_path=lib_path)
        self.eng.load(peers)
        self.eng.bind_routes(self.in_pos, self.out_pos)
        nb = self.eng.space_bytes(1, self.positions, self.depth)
        self.spaces = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(2)]
        self.stream = torch.cuda.current_stream()
        self.pop = OraclePopulation(peers, self.S)
        self.inv = self._inverse()
        self.msgs = np.zeros(0, abi.MESSAGE)  # the oracle's view of the next inbox
        self.threads = threads
        self.k = 0
        self.stats = {"escalations": 0, "esc_reasons": {}, "reencoded": 0, "commits": 0, "ready": 0,
                      "msgs": 0, "injected": 0}

    def _inverse(self):
        """mailbox position -> (receiving peer, sender slot), as arrays."""
        peer = np.full(self.positions, -1, np.int64)
        slot = np.full(self.positions, -1, np.int64)
        for j in range(self.S):
            ok = self.in_pos[j] != 0xFFFFFFFF
            p = np.nonzero(ok)[0]
            peer[self.in_pos[j, ok].astype(np.int64)] = p
            slot[self.in_pos[j, ok].astype(np.int64)] = j
        return peer, slot

    def export(self):
        return self.pop.export()

    def inject(self, idx, recs):
        """Host-side state edits on both sides (config 5's leader changes)."""
        idx = np.asarray(idx, np.int64)
        if len(idx):
            self.pop.reload(idx, recs)
            self.eng.load_peers(idx.astype(np.uint32), recs)
            self.stats["injected"] += len(idx)

    def _encode(self, msgs, space):
        """Write inbox records (receiver peer, sender slot) into a device space."""
        from dragonboat_amd.engine import load_library
        lib = self.eng.lib
        buf = np.zeros(self.eng.space_bytes(1, self.positions, self.depth), np.uint8)
        pos = self.in_pos[msgs["slot"].astype(np.int64), msgs["peer"].astype(np.int64)].astype(np.uint32)
        assert np.all(pos != 0xFFFFFFFF)
        order = np.argsort(pos, kind="stable")  # arrival order kept inside a mailbox
        m, pos = np.ascontiguousarray(msgs[order]), np.ascontiguousarray(pos[order])
        rc = lib.gr_space_encode(buf.ctypes.data, 1, self.positions, self.depth, m.ctypes.data if len(m) else None,
                                 len(m), pos.ctypes.data if len(pos) else None)
        assert rc == 0, rc
        import torch
        space.copy_(torch.from_numpy(buf))

    def override_inbox(self, msgs):
        """Replace the next pass's inbox (both sides) with inbox records."""
        msgs = np.asarray(msgs, abi.MESSAGE)
        self._encode(msgs, self.spaces[self.k % 2])
        self.msgs = msgs

    def step(self, loc, drop_fn=None):
        import torch
        k = self.k
        loc = np.asarray(loc, abi.LOCAL)
        self.eng.set_locals(loc)
        dev0 = self.eng.sync(self.n)
        src, dst = self.spaces[k % 2], self.spaces[(k + 1) % 2]
        self.eng.step_device(src.data_ptr(), dst.data_ptr(), 1, self.positions, 1, self.positions, self.n,
                             self.stream.cuda_stream, depth=self.depth)
        torch.cuda.synchronize()
        res = self.eng.collect_results(self.n)
        lim = parity.limits_from(res, self.n)
        o = self.pop.step(self.msgs, loc, lim, dev_before=dev0, threads=self.threads)
        dev = self.eng.sync(self.n)
        bad = parity.compare_states(dev, o["mid"], self.S)
        assert not bad, f"pass {k}: state {bad[:3]}"
        got = decode_space(dst.cpu().numpy(), 1, self.positions, self.depth)
        pos = got["peer"].astype(np.int64)
        got["peer"] = self.inv[0][pos].astype(np.uint32)
        got["slot"] = self.inv[1][pos].astype(np.uint8)
        want_prefix = self._route(parity.prefix_msgs(o, lim))
        bad = parity.compare_msgs(got, want_prefix)
        assert not bad, f"pass {k}: mailboxes {bad[:3]}"
        bad = parity.compare_results(res, o["results"])
        assert not bad, f"pass {k}: results {bad[:3]}"
        bad = parity.check_escalations(res, o["esc_mask"])
        assert not bad, f"pass {k}: unjustified escalations {bad[:3]}"
        esc = res[res["escalation"] != 0]
        st = self.stats
        st["escalations"] += len(esc)
        for r in esc:
            nm = abi.ESC_NAMES[r["escalation"]]
            st["esc_reasons"][nm] = st["esc_reasons"].get(nm, 0) + 1
        st["commits"] += int(np.sum(dev["committed"] > dev0["committed"]))
        st["ready"] += int(res["n_ready"].sum())
        st["msgs"] += len(got)
        full = self.pop.export()
        assert self.pop.representable().all(), "a peer outgrew its gr_peer record"
        nxt = self._route(o["msgs"])
        n_full = len(nxt)
        if drop_fn is not None:
            nxt = drop_fn(k, nxt)
        if len(esc) or len(nxt) != n_full:
            if len(esc):  # the host ran their suffix: reload them from the oracle
                idx = esc["peer"].astype(np.int64)
                self.eng.load_peers(idx.astype(np.uint32), full[idx])
            self._encode(nxt, dst)
            st["reencoded"] += 1
        self.msgs = nxt
        self.k += 1
        return res

    def _route(self, out):
        return route(out, self, self.G, self.R)

    def close(self):
        self.eng.close()
