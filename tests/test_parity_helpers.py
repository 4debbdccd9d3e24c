"""The parity helpers catch what they must: a one-field change in a state,
message or result record is reported (the vectorised screens only skip
records that are exactly equal)."""
import numpy as np

from dragonboat_amd import abi, populations as P
import parity


def test_state_field_change_is_reported():
    a = P.make_groups(50, 3, seed=1)
    b = a.copy()
    assert parity.compare_states(a, b, 3) == []
    b["committed"][7] += 1
    b["remotes"][11]["next"][2] += 1
    bad = parity.compare_states(a, b, 3)
    assert [p for p, _ in bad] == [7, 11]


def test_message_order_within_mailbox_matters():
    m = np.zeros(4, abi.MESSAGE)
    m["peer"] = [1, 1, 2, 1]
    m["slot"] = [0, 0, 1, 2]
    m["log_index"] = [10, 11, 5, 7]
    shuffled = m[[2, 3, 0, 1]]  # other mailboxes interleaved: same per-mailbox order
    assert parity.compare_msgs(m, shuffled) == []
    swapped = m[[1, 0, 2, 3]]   # two messages of mailbox (1, 0) swapped
    assert parity.compare_msgs(m, swapped)


def test_result_field_change_is_reported():
    r = np.zeros(5, abi.RESULT)
    r["peer"] = np.arange(5)
    o = r.copy()
    assert parity.compare_results(r, o) == []
    o["n_ready"][3] = 1
    o["ready"][3][0]["index"] = 9
    assert [p for p, _ in parity.compare_results(r, o)] == [3]


def test_escalation_predicate(built):
    """The oracle's escalation predicate (batch.cpp) justifies an escalation only
    when the item needs the host: a steady leader's ReplicateResp does not, a
    follower whose election timeout fires with committed <= applied does
    (ELECTION), a second reset in one pass does (RANDOM), a message past GR_C
    in one mailbox does (CAPACITY)."""
    import numpy as np
    from dragonboat_amd import abi, populations as P
    from oracle.pyoracle import OraclePopulation
    import parity
    G, R = 4, 3
    peers = P.make_groups(G, R, seed=3)
    topo = P.Topology(G, R)
    pop = OraclePopulation(peers, R)
    o = pop.step(None, P.propose_locals(R * G, np.arange(G), pass_index=0))
    msgs = topo.route_messages(o["msgs"])
    pop = OraclePopulation(peers, R)
    o = pop.step(None, P.propose_locals(R * G, np.arange(G), pass_index=0))
    # pass 2: claim the leader of group 0 escalated its first ack (item 0)
    loc = P.propose_locals(R * G, np.arange(G), pass_index=1)
    lim = np.full(R * G, 0xFFFFFFFF, np.uint32)
    lim[0] = 0
    o = pop.step(msgs, loc, lim, dev_before=pop.export())
    res = np.zeros(1, abi.RESULT)
    res["peer"], res["escalation"], res["esc_item"] = 0, abi.ESC_NAMES.index("capacity"), 0
    bad = parity.check_escalations(res, o["esc_mask"])
    assert bad and bad[0][2] == "capacity" and bad[0][3] == [], bad
    # a follower's election timeout with committed <= applied: ELECTION is justified
    p2 = peers.copy()
    f = G  # replica 1 of group 0
    p2["election_tick"][f] = p2["randomized_election_timeout"][f] - 1
    pop = OraclePopulation(p2, R)
    loc = P.propose_locals(R * G, [], pass_index=0, ticks=1)
    lim = np.full(R * G, 0xFFFFFFFF, np.uint32)
    lim[f] = 0
    o = pop.step(None, loc, lim, dev_before=p2)
    assert (int(o["esc_mask"][f]) >> abi.ESC_NAMES.index("election")) & 1
    assert not (int(o["esc_mask"][f]) >> abi.ESC_NAMES.index("capacity")) & 1
    # GR_C + 2 Heartbeats into one depth-GR_C mailbox: item GR_C is a CAPACITY item
    hb = np.zeros(abi.GR_C + 2, abi.MESSAGE)
    hb["peer"], hb["type"], hb["slot"], hb["term"] = f, abi.HEARTBEAT, 0, p2["term"][f]
    pop = OraclePopulation(peers, R)
    lim[f] = abi.GR_C
    o = pop.step(hb, None, lim, dev_before=peers)
    assert (int(o["esc_mask"][f]) >> abi.ESC_NAMES.index("capacity")) & 1
