"""The compact boundary (gr_step_compact, gpuraft.h gr_cmsg/gr_clocal/gr_cresult):
the C-ABI path a Go step worker calls, with the steady state's messages in 24 B
instead of 80, two per record where a mailbox's pair repeats itself (GR_CM_PAIR),
and results in 24 B instead of 168.

CPU: gr_pack_messages / gr_pair_messages / gr_unpack_messages / gr_pack_locals
are exact inverses on every message shape the engine and the oracle produce (a
record that does not fit its compact form travels in full as an ext record).
GPU: the compact path against the oracle after every pass (the Lockstep of
tests/simulate.py with GpuCompactBackend): steady state, leader churn, ticks +
ReadIndex (heartbeats with contexts, ReadyToRead: ext records both ways), BASELINE
config 3's shape and terms straddling 2^32.
"""
import ctypes

import numpy as np
import pytest

from dragonboat_amd import abi, populations as P
import simulate as SIM


def _lib():
    from dragonboat_amd.engine import load_library
    return load_library()


def _pack(lib, msgs):
    c = np.zeros(len(msgs), abi.CMSG)
    ext = np.zeros(len(msgs), abi.MESSAGE)
    nx = ctypes.c_size_t()
    assert lib.gr_pack_messages(msgs.ctypes.data, len(msgs), c.ctypes.data, ext.ctypes.data, ctypes.byref(nx)) == 0
    return c, ext[:nx.value].copy()


def _unpack(lib, c, ext):
    lib.gr_cmsg_count.restype = ctypes.c_size_t
    out = np.zeros(int(lib.gr_cmsg_count(c.ctypes.data, len(c))), abi.MESSAGE)
    assert lib.gr_unpack_messages(c.ctypes.data, len(c), ext.ctypes.data if len(ext) else None, len(ext),
                                  out.ctypes.data) == 0
    return out


def _random_messages(n, rng):
    m = np.zeros(n, abi.MESSAGE)
    m["peer"] = rng.integers(0, 1000, n)
    m["slot"] = rng.integers(0, 3, n)
    m["type"] = rng.choice([abi.REPLICATE, abi.REPLICATE_RESP, abi.HEARTBEAT, abi.HEARTBEAT_RESP, abi.NOOP,
                            abi.TIMEOUT_NOW, abi.READ_INDEX_RESP, abi.PROPOSE], n)
    wide = rng.random(n) < 0.1
    m["term"] = np.where(wide, rng.integers(2**32 - 3, 2**32 + 3, n, dtype=np.uint64),
                         rng.integers(0, 50, n, dtype=np.uint64))
    m["log_index"] = rng.choice([0, 5, 2**32 + 7, 2**63], n).astype(np.uint64) + rng.integers(0, 9, n, dtype=np.uint64)
    lt = rng.random(n)
    m["log_term"] = np.where(lt < 0.5, m["term"], np.where(lt < 0.8, 0, m["term"] - np.uint64(1)))
    c = rng.random(n)
    d = rng.choice([0, 1, 2**31 - 1, 2**31, 2**40], n).astype(np.uint64)
    m["commit"] = np.where(c < 0.4, m["log_index"] + d, np.where(c < 0.6, 0, m["log_index"] - d))
    h = rng.random(n)
    m["hint"] = np.where(h < 0.7, 0, m["log_index"] + rng.integers(0, 100, n, dtype=np.uint64))
    m["hint_high"] = np.where(rng.random(n) < 0.8, 0, rng.integers(1, 2**63, n, dtype=np.uint64))
    m["reject"] = rng.random(n) < 0.2
    ne = rng.choice([0, 1, 1, 2, 7], n)
    m["n_entries"] = ne
    two = (ne >= 2) & (rng.random(n) < 0.5)
    m["n_runs"] = np.where(ne == 0, 0, np.where(two, 2, 1))
    m["run2_offset"] = np.where(two, 1, 0)
    m["run_term"][:, 0] = np.where(ne == 0, 0, np.where(rng.random(n) < 0.8, m["term"], m["term"] - np.uint64(1)))
    m["run_term"][:, 1] = np.where(two, m["term"], 0)
    return m


def test_pack_round_trip(built):
    """unpack(pack(m)) == m byte for byte; steady-state shapes are compact."""
    lib = _lib()
    rng = np.random.default_rng(1)
    m = _random_messages(20000, rng)
    c, ext = _pack(lib, m)
    assert 0 < len(ext) < len(m)
    back = _unpack(lib, c, ext)
    assert back.tobytes() == m.tobytes()
    # every ext record is referenced once, in order
    x = (c["flags"] & abi.CM_EXT) != 0
    assert np.array_equal(c["aux"][x], np.arange(x.sum()))
    # the steady state fits: compact Replicates, accepting acks
    s = np.zeros(3, abi.MESSAGE)
    s["type"] = [abi.REPLICATE, abi.REPLICATE, abi.REPLICATE_RESP]
    s["term"] = 7
    s["log_index"] = 2**32 + 5
    s["log_term"][:2] = 7
    s["commit"][:2] = 2**32 + 4
    s["n_entries"][1], s["n_runs"][1], s["run_term"][1, 0] = 1, 1, 7
    c, ext = _pack(lib, s)
    assert len(ext) == 0 and _unpack(lib, c, ext).tobytes() == s.tobytes()


def _pair(lib, c):
    c = c.copy()
    n = ctypes.c_size_t()
    assert lib.gr_pair_messages(c.ctypes.data, len(c), ctypes.byref(n)) == 0
    return c[:n.value].copy()


def test_pair_round_trip(built):
    """GR_CM_PAIR: the steady state's mailbox pairs (a commit broadcast and the
    proposal after it at one LogIndex; two accepts at LogIndex, LogIndex + 1) merge
    into one record each and unpack to the same messages in order; anything else
    (other types, rejects, unequal fields, ext records, other mailboxes) stays
    single."""
    lib = _lib()
    rng = np.random.default_rng(4)
    n = 3000
    base = np.zeros(n, abi.MESSAGE)
    base["peer"] = rng.integers(0, 50, n)
    base["slot"] = rng.integers(0, 3, n)
    base["term"] = rng.integers(1, 4, n)
    base["log_index"] = rng.integers(2**32, 2**32 + 4, n, dtype=np.uint64)
    kind = rng.integers(0, 4, n)
    m = []
    for k in range(n):
        a = base[k].copy()
        if kind[k] == 0:  # Replicate pair: empty commit broadcast + one-entry proposal
            a["type"], a["log_term"], a["commit"] = abi.REPLICATE, a["term"], a["log_index"] - np.uint64(1)
            b = a.copy()
            b["n_entries"], b["n_runs"], b["run_term"][0] = 1, 1, a["term"]
            if rng.random() < 0.2:
                b["commit"] += np.uint64(1)  # unequal Commit: no pair
            m += [a, b]
        elif kind[k] == 1:  # accept pair
            a["type"] = abi.REPLICATE_RESP
            b = a.copy()
            b["log_index"] += np.uint64(1 if rng.random() < 0.8 else 2)
            m += [a, b]
        elif kind[k] == 2:  # reject + accept: no pair
            a["type"], a["reject"], a["hint"] = abi.REPLICATE_RESP, 1, a["log_index"]
            b = a.copy()
            b["reject"], b["hint"], b["log_index"] = 0, 0, a["log_index"] + np.uint64(1)
            m += [a, b]
        else:  # a heartbeat and a wide-term Replicate (ext): single
            a["type"], a["commit"] = abi.HEARTBEAT, a["log_index"]
            b = base[k].copy()
            b["type"], b["term"] = abi.REPLICATE, 2**32 + 1
            m += [a, b]
    msgs = np.array(m, abi.MESSAGE)
    c, ext = _pack(lib, msgs)
    cp = _pair(lib, c)
    pairs = (cp["flags"] & abi.CM_PAIR) != 0
    assert 0 < pairs.sum() < len(cp) < len(c)
    assert len(c) - len(cp) == pairs.sum()
    assert _unpack(lib, cp, ext).tobytes() == msgs.tobytes()
    # only Replicates and accepts pair; ENTRY2 only on a pair
    assert set(np.unique(cp["type"][pairs])) <= {abi.REPLICATE, abi.REPLICATE_RESP}
    assert not np.any((cp["flags"] & abi.CM_ENTRY2 != 0) & ~pairs)
    assert not np.any(pairs & ((cp["flags"] & (abi.CM_REJECT | abi.CM_EXT)) != 0))


def test_pack_locals_round_trip(built):
    lib = _lib()
    rng = np.random.default_rng(2)
    n = 5000
    loc = np.zeros(n, abi.LOCAL)
    loc["peer"] = rng.integers(0, 100, n)
    loc["ticks"] = rng.choice([0, 1, 3, 70000], n)
    loc["quiesced_ticks"] = rng.choice([0, 1, 300], n)
    loc["propose_entries"] = rng.integers(0, 5, n)
    loc["read_index"] = rng.random(n) < 0.2
    loc["read_ctx_low"] = np.where(loc["read_index"], rng.integers(1, 2**63, n, dtype=np.uint64), 0)
    loc["propose_has_config_change"] = rng.random(n) < 0.05
    loc["rand"] = rng.integers(0, 2**63, n, dtype=np.uint64)
    c = np.zeros(n, abi.CLOCAL)
    ext = np.zeros(n, abi.LOCAL)
    nx = ctypes.c_size_t()
    assert lib.gr_pack_locals(loc.ctypes.data, n, c.ctypes.data, ext.ctypes.data, ctypes.byref(nx)) == 0
    x = (c["flags"] & abi.CL_EXT) != 0
    assert x.sum() == nx.value and 0 < nx.value < n
    assert ext[c["ext"][x]].tobytes() == loc[x].tobytes()
    y = ~x
    for f in ("peer", "propose_entries", "ticks", "quiesced_ticks", "rand"):
        assert np.array_equal(c[f][y].astype(np.uint64), loc[f][y].astype(np.uint64)), f
    assert np.array_equal((c["flags"][y] & abi.CL_CONFIG_CHANGE) != 0, loc["propose_has_config_change"][y] != 0)


def _sim(G, passes, seed, R=3, locals_fn=None, inject_p=0.0, peers=None, drop_fn=None, halves=False, **mk):
    peers = P.make_groups(G, R, seed=seed, **mk) if peers is None else peers
    topo = P.Topology(G, R)
    rng = np.random.default_rng(seed)
    lf = locals_fn or (lambda k: P.propose_locals(R * G, np.arange(G), pass_index=k))
    inj = (lambda k, cur: P.inject_leader_change(cur, topo, inject_p, rng)) if inject_p else None
    backend = SIM.GpuCompactHalvesBackend if halves else SIM.GpuCompactBackend
    return SIM.simulate(backend, peers, topo, passes, lf, inject_fn=inj, slots=R, drop_fn=drop_fn)


@pytest.mark.gpu
def test_compact_steady_and_churn(gpu):
    st = _sim(1000, 6, seed=3)
    assert st["escalations"] == 0 and st["commits"] > 0
    st = _sim(500, 14, seed=5, inject_p=0.1)
    assert st["commits"] > 0


@pytest.mark.gpu
def test_compact_ticks_read_index_and_wide_terms(gpu):
    G, R = 256, 3
    rng = np.random.default_rng(9)

    def lf(k):
        loc = P.propose_locals(R * G, np.arange(G), pass_index=k)
        loc["ticks"] = rng.integers(0, 3, R * G)
        loc["read_index"] = rng.random(R * G) < 0.3
        loc["read_ctx_low"] = rng.integers(1, 2**63, R * G, dtype=np.uint64)
        loc["read_ctx_high"] = k
        return loc
    st = _sim(G, 10, seed=7, locals_fn=lf, check_quorum=True)
    assert st["ready"] > 0
    peers = P.make_groups(G, R, seed=8)
    peers["term"] = 2**32 - 1 + (np.arange(len(peers)) % 3)  # terms at and past 2^32
    _sim(G, 6, seed=8, peers=peers, inject_p=0.2)


@pytest.mark.gpu
def test_compact_config3(gpu):
    R, G = 5, 1000
    peers, active = P.config3(G, R)
    rng = np.random.default_rng(33)
    st = _sim(G, 8, seed=33, R=R, peers=peers, locals_fn=lambda k: P.config3_locals(G, R, active, k),
              drop_fn=lambda k, m: P.drop_acks(m, 0.1, rng))
    assert st["ready"] > 0


@pytest.mark.gpu
def test_compact_halves(gpu):
    """gr_step_compact_begin + _end (the pipelined host path of bench.py) equal the
    oracle after every pass like gr_step_compact, and refuse misuse: _end without a
    _begin, a second _begin before its _end (GR_EINVAL, nothing run)."""
    st = _sim(600, 8, seed=7, inject_p=0.1, halves=True)
    assert st["commits"] > 0
    from dragonboat_amd.engine import Engine
    eng = Engine(64 * 3, 3)
    eng.load(P.make_groups(64, 3, seed=1))
    ob = abi.COutbox()
    assert eng.lib.gr_step_compact_end(eng._h, ctypes.byref(ob)) == -1  # GR_EINVAL
    cm, xm = eng.pack_messages(np.zeros(0, abi.MESSAGE))
    cl, xl = eng.pack_locals(P.propose_locals(64 * 3, np.arange(64), pass_index=0))
    ib = abi.cinbox_of(cm, xm, cl, xl)
    before = eng.sync_peers(np.arange(4))
    assert eng.lib.gr_step_compact_begin(eng._h, ctypes.byref(ib)) == 0
    assert eng.lib.gr_step_compact_begin(eng._h, ctypes.byref(ib)) == -1
    # between _begin and _end the pending pass owns the scratch and lane rows:
    # every entry point that would use them refuses (GR_ESTATE), nothing written
    ESTATE = -6
    sl = np.arange(4, dtype=np.uint32)
    pe = P.make_groups(64, 3, seed=2)[:4]
    assert eng.lib.gr_load_peers(eng._h, sl.ctypes.data, pe.ctypes.data, 4) == ESTATE
    assert eng.lib.gr_load_groups(eng._h, 0, pe.ctypes.data, 4) == ESTATE
    assert eng.lib.gr_sync_peers_to_host(eng._h, sl.ctypes.data, pe.ctypes.data, 4) == ESTATE
    ap = np.zeros(4, np.uint64)
    assert eng.lib.gr_notify_applied(eng._h, sl.ctypes.data, ap.ctypes.data, 4) == ESTATE
    assert eng.lib.gr_compact_log(eng._h, sl.ctypes.data, ap.ctypes.data, 4, None) == ESTATE
    loc = P.propose_locals(64 * 3, np.arange(64), pass_index=1)
    assert eng.lib.gr_set_locals(eng._h, loc.ctypes.data, len(loc)) == ESTATE
    sib = abi.inbox_of(np.zeros(0, abi.MESSAGE), loc)
    sob = abi.Outbox()
    assert eng.lib.gr_step(eng._h, ctypes.byref(sib), ctypes.byref(sob)) == ESTATE
    res = np.zeros(4, abi.RESULT)
    assert eng.lib.gr_collect_results(eng._h, 0, res.ctypes.data, 4) == ESTATE
    assert eng.lib.gr_step_compact_end(eng._h, ctypes.byref(ob)) == 0
    assert ob.n_results == 64 * 3 or ob.n_results == 64  # a result per lane with input
    assert eng.lib.gr_release_coutbox(eng._h, ctypes.byref(ob)) == 0
    # the refused load wrote nothing (slots 0..3 are as the pass left them, which
    # differs from `pe`), and after _end the engine takes calls again
    after = eng.sync_peers(np.arange(4))
    assert after.tobytes() != pe.tobytes() and after["node_id"].tobytes() == before["node_id"].tobytes()
    eng.load_peers(np.arange(4), after)
    eng.close()

