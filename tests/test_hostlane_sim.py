"""The kernel's lane code (gr_lane.h, built for the host as tests/_build/libhostlane.so)
against the oracle, bit-exact after every pass. The same code runs on the GPU
in tests/test_gpu.py; these CPU runs pin the logic without a device."""
import numpy as np
import pytest

from dragonboat_amd import abi, populations as P
import simulate as SIM


def _run(G, passes, seed, locals_fn=None, inject_p=0.0, **mk):
    R = 3
    peers = P.make_groups(G, R, seed=seed, **mk)
    topo = P.Topology(G, R)
    rng = np.random.default_rng(seed)
    lf = locals_fn or (lambda k: P.propose_locals(R * G, np.arange(G), pass_index=k))
    inj = (lambda k, cur: P.inject_leader_change(cur, topo, inject_p, rng)) if inject_p else None
    return SIM.simulate(SIM.HostlaneBackend, peers, topo, passes, lf, inject_fn=inj)


def test_steady_state_commit(built):
    """BASELINE config 2 shape: leader commits one index per pass after warm-up.
    The lean steady-state lane (gr_fast.h) must finish almost every lane."""
    from oracle.pyoracle import hostlane_counters, hostlane_steady_lanes
    f0, b0 = hostlane_counters()
    s0 = hostlane_steady_lanes()
    st = _run(64, 6, seed=3)
    f1, b1 = hostlane_counters()
    assert st["escalations"] == 0
    assert st["commits"] > 0
    fast, bailed = f1 - f0, b1 - b0
    assert fast > 0 and bailed <= fast // 4, (fast, bailed)
    # the closed-form steady lanes (gr_steady.h) finished lanes of both roles'
    # steady waves, checked against the oracle like every other lane
    assert hostlane_steady_lanes() - s0 > 0


def test_leader_change_churn(built):
    """BASELINE config 5 shape: rejects, decreaseTo, conflict truncation; the
    general lane steps the follower side of the hand-overs -- step-downs, term
    adoptions, truncating merges, lookups below the newest run -- checked
    against the oracle like every other lane."""
    from oracle.pyoracle import hostlane_counters
    _, b0 = hostlane_counters()
    st = _run(200, 20, seed=5, inject_p=0.1)
    assert st["commits"] > 0
    _, b1 = hostlane_counters()
    assert b1 > b0


@pytest.mark.parametrize("inject_p", [0.0, 0.1])
def test_unhinted_waves_lane_closed_form(built, inject_p):
    """Every wave unhinted in a split pass (as in a pass's first passes, or waves
    whose groups' leaders sit on different replicas): the steady kernel's LC
    instance runs each lane's own role's closed form (gr_steady.h
    lane_closed_form, the slot from the header), the rest FastLane by role and
    the general lane; steady state and config-5 churn, bit-exact with the
    oracle after every pass, and the closed forms did finish lanes."""
    from oracle.pyoracle import hostlane_lib, hostlane_steady_lanes
    hl = hostlane_lib()
    hl.hl_force_unhinted(1)
    try:
        s0 = hostlane_steady_lanes()
        st = _run(128, 10, seed=7, inject_p=inject_p)
        assert st["commits"] > 0
        assert hostlane_steady_lanes() - s0 > 0
    finally:
        hl.hl_force_unhinted(0)


def test_forwarded_proposals(built):
    """ProposeEntries on every replica: followers forward (handleFollowerPropose,
    raft.go:1346-1357) and the leader appends the forwarded batches on the device
    (handleLeaderPropose :1125-1146), reported as n_forwarded/forwarded_entries
    with propose_first at the first of them. A forwarded batch holding a config
    change escalates CONFIG_CHANGE; leader churn mixes in stepped-down leaders."""
    G, R = 120, 3

    def lf(k):
        rng = np.random.default_rng([7, k])
        loc = P.propose_locals(R * G, np.arange(R * G), pass_index=k)
        loc["propose_entries"] = rng.integers(1, 4, R * G)
        loc["propose_has_config_change"] = rng.random(R * G) < 0.02
        return loc
    st = _run(G, 10, seed=9, locals_fn=lf, inject_p=0.05)
    assert st["forwarded"] > G, st
    # (12 of 120 groups over 10 passes with 6-deep mailboxes: more of each churn
    # pass's messages reach the lane before an escalation stops it)
    assert "unsupported" not in st["esc_reasons"] or st["esc_reasons"]["unsupported"] <= G // 8, st
    assert st["esc_reasons"].get("config_change", 0) > 0, st


@pytest.mark.parametrize("check_quorum", [False, True])
def test_ticks_and_read_index(built, check_quorum):
    """Tick sweep (heartbeats, election timeouts, checkQuorum) + leader ReadIndex."""
    G, R = 96, 3
    rng = np.random.default_rng(9)

    def lf(k):
        loc = P.propose_locals(R * G, np.arange(G), pass_index=k, ticks=1)
        loc["ticks"] = rng.integers(0, 3, R * G)
        ri = rng.random(R * G) < 0.3
        loc["read_index"] = ri
        loc["read_ctx_low"] = rng.integers(1, 2**63, R * G, dtype=np.uint64)
        loc["read_ctx_high"] = k
        loc["propose_entries"] = np.where(rng.random(R * G) < 0.5, loc["propose_entries"], 0)
        return loc
    st = _run(G, 12, seed=7, locals_fn=lf, check_quorum=check_quorum)
    assert st["msgs"] > 0


def test_wide_terms_escalate(built):
    """Terms >= 2^32 never enter a device mailbox (32-bit term fields): the sender
    escalates GR_ESC_WIDE_TERM, a host-encoded inbox message escalates at the
    receiver, and every applied item still matches the oracle bit for bit."""
    st = _run(32, 5, seed=4, term_lo=2**32 - 1, term_hi=2**32 + 2)
    assert st["esc_reasons"].get("wide_term", 0) > 0
    assert st["commits"] > 0  # groups whose terms still fit keep committing on the device


def _config3(backend, G, passes):
    R = 5
    peers, active = P.config3(G, R)
    topo = P.Topology(G, R)
    rng = np.random.default_rng(33)
    return SIM.simulate(backend, peers, topo, passes, lambda k: P.config3_locals(G, R, active, k),
                        slots=R, drop_fn=lambda k, m: P.drop_acks(m, 0.1, rng))


def test_config3_read_index_quiesced(built):
    """BASELINE config 3 shape (R=5): 90% quiesced groups (QuiescedTick only, the
    lean lane), 10% active with a ReadIndex per pass, heartbeat acks dropped
    with p=0.1, checkQuorum on half: bit-exact vs the oracle every pass."""
    from oracle.pyoracle import hostlane_counters, hostlane_tick_lanes
    f0, b0 = hostlane_counters()
    t0 = hostlane_tick_lanes()
    st = _config3(SIM.HostlaneBackend, 300, 10)
    f1, b1 = hostlane_counters()
    t1 = hostlane_tick_lanes()
    assert st["ready"] > 0  # ReadIndex confirmations reached ReadyToRead
    assert f1 - f0 > 0.8 * 300 * 5 * 10 * 0.9 * 0.9  # quiesced lanes stay on the lean lane
    # the active groups' heartbeat / ReadIndex / tick lanes mostly take the tick lane (gr_tick.h)
    assert t1 - t0 > 0.6 * (b1 - b0), (t1 - t0, b1 - b0)


def test_config1_single_group(built):
    """BASELINE config 1 shape: one group x 3 replicas, one 1-entry proposal per
    pass for 300 passes, committed traced against the oracle every pass."""
    st = _run(1, 300, seed=1)
    assert st["escalations"] == 0 and st["commits"] >= 290 * 3 - 10


def staggered_acks(G, R=3, seed=21):
    """Leaders three entries past committed with both followers' match at
    committed; follower 1 acks committed+1 and +2, follower 2 acks committed+3:
    three commit advances in one pass (the closed-form steady leader
    keeps two commit broadcasts and must hand this lane to FastLane)."""
    peers = P.make_groups(G, R, seed=seed)
    L = peers[:G]
    c = L["committed"].copy()
    for r in range(R):
        peers[r * G:(r + 1) * G]["last_index"] = c + np.uint64(3)
    L["remotes"]["next"][:, :R] = (c + np.uint64(4))[:, None]
    L["remotes"]["match"][:, 0] = c + np.uint64(3)  # self
    msgs = np.zeros(3 * G, abi.MESSAGE)
    for k, (slot, d) in enumerate(((1, 1), (1, 2), (2, 3))):
        m = msgs[k * G:(k + 1) * G]
        m["peer"] = np.arange(G, dtype=np.uint32)
        m["slot"] = slot
        m["type"] = abi.REPLICATE_RESP
        m["term"] = L["term"]
        m["log_index"] = c + np.uint64(d)
    order = np.lexsort((np.arange(len(msgs)), msgs["slot"], msgs["peer"]))
    return peers, msgs[order]


def test_steady_leader_staggered_acks(built):
    """Three commit advances in one pass on steady leaders (sync bits set at load,
    the device hint), with the device's hints and the split schedule: every
    lane, state and message equal to the oracle."""
    from oracle.pyoracle import hostlane_lib, hostlane_steady_lanes
    G, R = 128, 3
    peers, msgs = staggered_acks(G, R)
    hl = hostlane_lib()
    hl.hl_true_hints(1)
    try:
        ls = SIM.Lockstep(SIM.HostlaneBackend, peers, R)
        s0 = hostlane_steady_lanes()
        out, res = ls.step(msgs, np.zeros(0, abi.LOCAL))
        assert not np.any(res["escalation"])
        # the leaders committed all three (the median reached committed + 3)
        st = ls.export()
        assert np.all(st["committed"][:G] == peers["committed"][:G] + np.uint64(3))
        # three commit broadcasts per follower this pass
        assert len(out[(out["peer"] < G) & (out["type"] == abi.REPLICATE)]) == 3 * 2 * G
        ls.close()
        assert hostlane_steady_lanes() >= s0
    finally:
        hl.hl_true_hints(0)


def test_steady_leaders_stay_closed_form(built):
    """BASELINE config 2/4 steady state with the device's hints: after the first
    passes set the sync bits (H_NX, H_MS, H_MP: match = lastIndex - 2 in the
    pipelined steady state), every leader pass is the closed form SteadyLeader
    (gr_steady.h), with no MATCH row loaded, and parity holds every pass. Guards the
    header bits' steady-state values: a wrong one keeps every test green but sends
    the headline's leaders through FastLane."""
    from oracle.pyoracle import hostlane_lib, hostlane_steady_leaders
    G, R, passes, warm = 128, 3, 10, 4
    hl = hostlane_lib()
    hl.hl_true_hints(1)
    try:
        counts = []

        def lf(k):
            counts.append(hostlane_steady_leaders())
            return P.propose_locals(R * G, np.arange(G), pass_index=k)
        peers = P.make_groups(G, R, seed=11)
        st = SIM.simulate(SIM.HostlaneBackend, peers, P.Topology(G, R), passes, lf)
        counts.append(hostlane_steady_leaders())
        assert st["escalations"] == 0
        per_pass = np.diff(counts)[warm:]
        assert np.all(per_pass == G), per_pass
    finally:
        hl.hl_true_hints(0)
