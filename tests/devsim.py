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


def run_device(G, R, passes, placement="local", seed=2, tick_every=0, stats=None, inject_p=0.0, mix=False):
    """tick_every > 0: one Tick for every peer on passes k % tick_every == tick_every - 1
    (leader heartbeats and their acks: messages with cold fields).
    inject_p > 0: BASELINE config 5's leader changes (populations.inject_leader_change)
    before every pass after the first, on both sides, proposals on the current leaders.
    mix: peers in a group-major order (peer g*R + r), so every wave holds leaders
    and followers; the routes are then plain tables (local placement only)."""
    import torch
    S = R
    ex = Exchange(G, R, S, 1, 0, placement, seed=seed)
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
        ex.step(eng, spaces, k, stream)
        torch.cuda.synchronize()
        if placement == "spread" and stats is not None:  # cold-field entries the side buffers carried
            sb = len(ex.side[1]) // ex.n_chunks
            hdr = ex.side[1].cpu().numpy().reshape(ex.n_chunks, sb)[:, :4].copy().view(np.uint32)[:, 0]
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
        got = decode_space(raw, ex.n_chunks, ex.positions, ex.depth)
        for m in got:
            p, j = inv[int(m["peer"])]
            m["peer"], m["slot"] = p, j
        # oracle messages -> (receiver, sender slot) records in arrival order
        want = route(o["msgs"], ex, G, R, perm)
        bad = parity.compare_msgs(got, want)
        assert not bad, f"pass {k}: mailboxes {bad[:3]}"
        bad = parity.compare_results(res, o["results"])
        assert not bad, f"pass {k}: results {bad[:3]}"
        msgs = want
    final = eng.sync(n)
    eng.close()
    return final


def route(out, ex, G, R, perm=None):
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
