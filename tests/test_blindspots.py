"""Parity on populations the steady-state generators never build (VERDICT r01,
item 1): observers, single-voter groups, leader transfers in flight, leader
remotes in Snapshot state, terms straddling 2^32, the CheckQuorum step-down
(heartbeatTimeout 1 and 2), and ReadIndex from followers and observers.

Each workload runs through the engine -- libgpuraft.so on the GPU under -m gpu,
the host build of the same lane code on the CPU -- against the oracle after
every pass (state of every peer, every message, every result), and every
escalation must be one the oracle's own execution of that item justifies
(parity.check_escalations, the escalation predicate of oracle/batch.cpp).
"""
import numpy as np
import pytest

from dragonboat_amd import abi, populations as P
import simulate as SIM

BACKENDS = [pytest.param("cpu", id="hostlane"), pytest.param("gpu", id="gpu", marks=pytest.mark.gpu)]


def _backend(name, request):
    if name == "gpu":
        request.getfixturevalue("gpu")
        return SIM.GpuBackend
    request.getfixturevalue("built")
    return SIM.HostlaneBackend


def _locals(M, G, seed, prop=0.8, ri=0.2, tick=0.3, max_ticks=1, prop_everywhere=0.0):
    """locals_fn(k, state): proposals on current leaders (and on a fraction of the
    other members, which forward them), ReadIndex and ticks on random members."""
    n = M * G

    def lf(k, state):
        rng = np.random.default_rng([seed, k])
        lead = state["state"] == abi.LEADER
        loc = P.propose_locals(n, [], pass_index=k, seed=seed)
        want = (lead & (rng.random(n) < prop)) | (~lead & (rng.random(n) < prop_everywhere))
        loc["propose_entries"] = np.where(want, rng.integers(1, 3, n), 0)
        loc["read_index"] = rng.random(n) < ri
        loc["read_ctx_low"] = rng.integers(1, 2**63, n, dtype=np.uint64)
        loc["read_ctx_high"] = k + 1
        loc["ticks"] = np.where(rng.random(n) < tick, rng.integers(1, max_ticks + 1, n), 0)
        return loc
    return lf


@pytest.mark.parametrize("R,obs", [(2, 1), (3, 1), (3, 2), (5, 2)])
@pytest.mark.parametrize("be", BACKENDS)
def test_observers(be, R, obs, request):
    """Observer slots (raft.observers): leaders broadcast Replicates and
    heartbeats to them (raft.go:534-546, 575-587, observers only on a zero
    context), observers append and ack without voting, forward proposals and
    ReadIndex to the leader (handleObserverPropose/ReadIndex), and receive
    ReadIndexResp (raft.go:1391-1399); leader churn among the voters."""
    M, G = R + obs, 150
    peers = P.make_groups(G, R, seed=40 + R + obs, observers=obs)
    topo = P.Topology(G, M)
    rng = np.random.default_rng(R * 10 + obs)
    st = SIM.simulate(_backend(be, request), peers, topo, 10, _locals(M, G, 41, prop_everywhere=0.1), slots=M,
                      inject_fn=lambda k, cur: P.inject_leader_change(cur, topo, 0.05, rng))
    fin = st["final"].reshape(M, G)
    assert st["ready"] > 0 and st["commits"] > 0
    # observers followed the log (their committed advanced from the start)
    start = peers.reshape(M, G)["committed"]
    assert np.all(fin["committed"][R:] >= start[R:]) and np.any(fin["committed"][R:] > start[R:])


@pytest.mark.parametrize("obs", [0, 1])
@pytest.mark.parametrize("be", BACKENDS)
def test_single_voter(be, obs, request):
    """Single-voter groups (quorum 1): a proposal commits at once (appendEntries ->
    tryCommit, raft.go:643-654), a local ReadIndex is ready at once and an
    observer's is answered at once (handleLeaderReadIndex single-node branch,
    raft.go:1171-1203, TestLeaderReadIndexOnSingleNodeCluster,
    TestObserverCanReadIndexQuorum1)."""
    M, G = 1 + obs, 200
    peers = P.make_groups(G, 1, seed=50 + obs, observers=obs)
    topo = P.Topology(G, M)
    st = SIM.simulate(_backend(be, request), peers, topo, 8, _locals(M, G, 51, ri=0.5), slots=M)
    assert st["commits"] > 0 and st["ready"] > 0


def _transfer_requests(topo, p, seed):
    """extra_fn: RequestLeaderTransfer(target) delivered at random members
    (peer.go:116-124: From = Hint = target); followers forward it to the leader."""
    G, M = topo.G, topo.R

    def ex(k, state):
        rng = np.random.default_rng([seed, k])
        out = []
        for g in np.nonzero(rng.random(G) < p)[0]:
            at = int(rng.integers(0, M))
            tgt = int(rng.integers(0, M))
            m = np.zeros(1, abi.MESSAGE)[0]
            m["peer"] = at * G + g
            m["type"] = abi.LEADER_TRANSFER
            m["slot"] = tgt
            m["hint"] = tgt + 1
            out.append(m)
        return np.array(out, abi.MESSAGE) if out else None
    return ex


@pytest.mark.parametrize("be", BACKENDS)
def test_leader_transfer(be, request):
    """Leader transfer in flight: TimeoutNow when the target's ack catches it up
    (raft.go:1216-1219, the target then campaigns on the host), proposals dropped
    while transferring (raft.go:1130-1133), the transfer aborted after
    electionTimeout ticks (leaderTick, raft.go:403-429,
    TestLeaderTransferTimeout), and RequestLeaderTransfer messages at leaders and
    followers (handleLeaderLeaderTransfer :1242-1262, follower forward :1380-1389)."""
    M, G = 3, 200
    peers = P.make_groups(G, 3, seed=60, election=4)
    topo = P.Topology(G, M)
    rng = np.random.default_rng(61)

    def inject(k, cur):
        return P.inject_leader_transfer(cur, topo, 0.15 if k % 3 == 0 else 0.0, rng)
    st = SIM.simulate(_backend(be, request), peers, topo, 12, _locals(M, G, 62, tick=0.5), slots=M,
                      inject_fn=inject, extra_fn=_transfer_requests(topo, 0.05, 63))
    assert st["commits"] > 0
    assert st["esc_reasons"].get("unsupported", 0) > 0, st["esc_reasons"]  # TimeoutNow reached targets


@pytest.mark.parametrize("be", BACKENDS)
def test_snapshot_state_remotes(be, request):
    """Leader remotes in Snapshot state: paused (no Replicate sent, isPaused
    remote.go:158-171) until an accepted ack with match >= snapshotIndex moves
    them to Retry (respondedTo, remote.go:130-138); acks below snapshotIndex keep
    them paused; heartbeat acks of Snapshot remotes."""
    M, G = 3, 200
    peers = P.make_groups(G, 3, seed=70)
    topo = P.Topology(G, M)
    rng = np.random.default_rng(71)
    st = SIM.simulate(_backend(be, request), peers, topo, 10, _locals(M, G, 72, ri=0.1, tick=0.2), slots=M,
                      inject_fn=lambda k, cur: P.inject_snapshot_state(cur, topo, 0.3, rng))
    fin = st["final"].reshape(M, G)
    assert st["commits"] > 0
    # acks at or above snapshotIndex moved Snapshot remotes to Retry on the device
    assert st["snapshot_left"] > 0, st
    assert np.any(fin["remotes"]["state"][0] == abi.RETRY) or np.any(fin["remotes"]["state"][0] == abi.WAIT)


@pytest.mark.parametrize("be", BACKENDS)
def test_terms_straddling_2_32(be, request):
    """Terms crossing 2^32 under leader churn: messages whose terms reach 2^32
    never enter a 32-bit device mailbox (GR_ESC_WIDE_TERM at the sender, MT_WIDE at
    a host-encoded receiver); groups below it keep running on the device."""
    M, G = 3, 200
    peers = P.make_groups(G, 3, seed=80, term_lo=2**32 - 3, term_hi=2**32 - 1)
    topo = P.Topology(G, M)
    rng = np.random.default_rng(81)
    # one churn wave (terms T -> T+1 cross 2^32 for T = 2^32-1); repeated churn of
    # one group could make a lagging log need Replicates of more than two term
    # runs, which gr_message records cannot carry (the host keeps those)
    st = SIM.simulate(_backend(be, request), peers, topo, 10, _locals(M, G, 82, tick=0.2), slots=M,
                      inject_fn=lambda k, cur: P.inject_leader_change(cur, topo, 0.7 if k == 1 else 0.0, rng))
    assert st["esc_reasons"].get("wide_term", 0) > 0, st["esc_reasons"]
    assert st["commits"] > 0


@pytest.mark.parametrize("ht", [1, 2])
@pytest.mark.parametrize("be", BACKENDS)
def test_check_quorum_step_down(be, ht, request):
    """CheckQuorum: a leader whose remotes stayed inactive for electionTimeout
    ticks steps down (leaderHasQuorum, raft.go:262-271, 1117-1123;
    TestLeaderStepdownWhenQuorumLost), one that hears acks stays
    (TestLeaderStepdownWhenQuorumActive); the same tick's heartbeat quirk: after
    the step-down reset, heartbeatTick++ reaches heartbeatTimeout only when it
    is 1 (then reset to 0, handled by the follower table), else stays 1.
    Some of the stepping-down leaders are transferring (abort in the same tick)."""
    M, G = 3, 200
    ET = 5  # config.Validate: ElectionRTT > 2 * HeartbeatRTT
    peers = P.make_groups(G, 3, seed=90 + ht, election=ET, heartbeat=ht, check_quorum=True)
    lead = peers[:G]
    rng = np.random.default_rng(91)
    lead["election_tick"] = rng.integers(0, ET, G)
    lost = rng.random(G) < 0.5
    rem = lead["remotes"]
    rem["active"][lost] = 0
    xfer = lost & (rng.random(G) < 0.3)
    lead["leader_transfer_target"][xfer] = 2
    topo = P.Topology(G, M)

    def lf(k, state):
        loc = P.propose_locals(M * G, [], pass_index=k, ticks=1)
        return loc

    def drop(k, msgs):  # the lost groups' leaders hear nothing
        to_lead = msgs["peer"] < G
        iso = lost[msgs["peer"] % G]
        return msgs[~(to_lead & iso)]
    st = SIM.simulate(_backend(be, request), peers, topo, 2 * ET + 2, lf, slots=M, drop_fn=drop)
    fin = st["final"].reshape(M, G)
    assert np.all(fin["state"][0][lost] != abi.LEADER)  # stepped down (or campaigned on the host)
