"""The reference's multi-node and tick/ReadIndex known-answer tests driven
through the engine: libgpuraft.so on the GPU under
-m gpu, the host build of the same lane code on the CPU. Each test restates one
reference test over tests/network.py (raft_etcd_test.go's in-memory network) or
over engine records built to the state the reference test constructs, asserts
the reference's expected values, and is compared with the oracle after every
pass (state, messages, results, escalation predicate). Four identical copies of
each group run side by side and must agree.

Payload bytes (Entry.Cmd) never reach the engine, so the reference's data
comparisons (nextEnts Cmd equality in TestLogReplication) are out of scope;
committed indexes, logs, messages and ReadyToRead are checked.
"""
import numpy as np
import pytest

from dragonboat_amd import abi
from network import Net, node_records
import simulate as SIM

BACKENDS = [pytest.param("cpu", id="hostlane"), pytest.param("gpu", id="gpu", marks=pytest.mark.gpu)]
COPIES = 4


def _backend(name, request):
    if name == "gpu":
        request.getfixturevalue("gpu")
        return SIM.GpuBackend
    request.getfixturevalue("built")
    return SIM.HostlaneBackend


def _committed(net, nid):
    c = net.all_copies(nid)["committed"]
    assert np.all(c == c[0]), f"copies of node {nid} disagree: {c}"
    return int(c[0])


def _election(net, nid):
    net.send(net.msg(nid, nid, abi.ELECTION))


def _propose(net, frm, to, n=1):
    net.send(net.msg(frm, to, abi.PROPOSE, entries=n))


# ---- raft_etcd_test.go:633-690 TestLogReplication
@pytest.mark.parametrize("be", BACKENDS)
@pytest.mark.parametrize("case", [0, 1])
def test_log_replication(be, case, request):
    net = Net(_backend(be, request), [1, 2, 3], copies=COPIES)
    _election(net, 1)
    if case == 0:
        _propose(net, 1, 1)
        want = 2
    else:
        _propose(net, 1, 1)
        net.send(net.msg(1, 2, abi.ELECTION))
        _propose(net, 1, 2)
        want = 4
    for nid in (1, 2, 3):
        assert _committed(net, nid) == want
        assert int(net.state(nid)["last_index"]) == want
    net.close()


# ---- raft_etcd_test.go:692-704 TestSingleNodeCommit
@pytest.mark.parametrize("be", BACKENDS)
def test_single_node_commit(be, request):
    net = Net(_backend(be, request), [1], copies=COPIES)
    _election(net, 1)
    _propose(net, 1, 1)
    _propose(net, 1, 1)
    assert _committed(net, 1) == 3
    net.close()


# ---- raft_etcd_test.go:707-747 TestCannotCommitWithoutNewTermEntry
@pytest.mark.parametrize("be", BACKENDS)
def test_cannot_commit_without_new_term_entry(be, request):
    net = Net(_backend(be, request), [1, 2, 3, 4, 5], copies=COPIES)
    _election(net, 1)
    for o in (3, 4, 5):
        net.cut(1, o)
    _propose(net, 1, 1)
    _propose(net, 1, 1)
    assert _committed(net, 1) == 1
    net.recover()
    net.ignore(abi.REPLICATE)  # avoid committing the new term's noop
    _election(net, 2)
    assert _committed(net, 2) == 1
    net.recover()
    net.send(net.msg(2, 2, abi.LEADER_HEARTBEAT))
    _propose(net, 2, 2)
    assert _committed(net, 2) == 5
    net.close()


# ---- raft_etcd_test.go:751-779 TestCommitWithoutNewTermEntry
@pytest.mark.parametrize("be", BACKENDS)
def test_commit_without_new_term_entry(be, request):
    net = Net(_backend(be, request), [1, 2, 3, 4, 5], copies=COPIES)
    _election(net, 1)
    for o in (3, 4, 5):
        net.cut(1, o)
    _propose(net, 1, 1)
    _propose(net, 1, 1)
    assert _committed(net, 1) == 1
    net.recover()
    _election(net, 2)
    assert _committed(net, 1) == 4
    net.close()


def fresh_leader(ids, voters, leader=1, election=10, heartbeat=1, check_quorum=False, copies=COPIES):
    """Records of newTestRaft nodes after the leader ran becomeCandidate() and
    becomeLeader() (raft.go:676-702) alone: term 1, its noop at index 1
    uncommitted, every remote reset (next 1, inactive), its own match 1."""
    peers = node_records(ids, set(voters), copies, election=election, heartbeat=heartbeat,
                         check_quorum=check_quorum)
    r = ids.index(leader)
    L = peers[r * copies:(r + 1) * copies]
    L["term"] = 1
    L["vote"] = leader
    L["state"] = abi.LEADER
    L["leader_id"] = leader
    L["last_index"] = 1
    L["n_runs"] = 2
    L["run_start"][:, 1] = 1
    L["run_term"][:, 1] = 1
    L["remotes"][:, r]["match"] = 1
    L["remotes"][:, r]["next"] = 2
    return peers


# ---- raft_etcd_test.go:1602-1634 TestLeaderStepdownWhenQuorumActive / Lost
@pytest.mark.parametrize("be", BACKENDS)
@pytest.mark.parametrize("active", [True, False])
def test_leader_stepdown_check_quorum(be, active, request):
    ET = 5
    net = Net(_backend(be, request), [1, 2, 3], copies=COPIES,
              records=fresh_leader([1, 2, 3], [1, 2, 3], election=ET, check_quorum=True))
    for _ in range(ET + 1):
        msgs = net.msg(2, 1, abi.HEARTBEAT_RESP, term=1) if active else None
        out = net.ls.step(msgs, net.locals_({1: {"ticks": 1}}))  # Handle(HeartbeatResp), then tick()
        net.ls.apply_all()
    st = net.all_copies(1)["state"]
    assert np.all(st == (abi.LEADER if active else abi.FOLLOWER)), st
    net.close()


# ---- raft_etcd_test.go:1951-2005 TestBcastBeat
@pytest.mark.parametrize("be", BACKENDS)
def test_bcast_beat(be, request):
    """A log restored from a snapshot at 1000 (term 1), leader at term 2 with its
    noop at 1001 and ten entries; a slow follower (match 5, next 6) and a caught-up
    one. LeaderHeartbeat sends exactly one Heartbeat to each, Commit =
    min(committed, match), no LogIndex/LogTerm/entries."""
    off = 1000
    ids = [1, 2, 3]
    peers = node_records(ids, set(ids), COPIES)
    L = peers[:COPIES]
    L["term"] = 2
    L["vote"] = 1
    L["state"] = abi.LEADER
    L["leader_id"] = 1
    L["committed"] = off
    L["applied"] = off
    L["first_index_m1"] = off
    L["last_index"] = off + 11
    L["n_runs"] = 2
    L["run_start"][:, 0], L["run_term"][:, 0] = off, 1
    L["run_start"][:, 1], L["run_term"][:, 1] = off + 1, 2
    rem = L["remotes"]
    rem["match"][:, 0], rem["next"][:, 0] = off + 11, off + 12
    rem["match"][:, 1], rem["next"][:, 1] = 5, 6
    rem["match"][:, 2], rem["next"][:, 2] = off + 11, off + 12
    for r in (1, 2):  # followers: same log, term 2
        F = peers[r * COPIES:(r + 1) * COPIES]
        F["term"], F["leader_id"], F["committed"], F["applied"], F["first_index_m1"] = 2, 1, off, off, off
        F["last_index"], F["n_runs"] = off + 11, 2
        F["run_start"][:, 0], F["run_term"][:, 0] = off, 1
        F["run_start"][:, 1], F["run_term"][:, 1] = off + 1, 2
        F["remotes"]["next"] = off + 12
    net = Net(_backend(be, request), ids, copies=COPIES, records=peers)
    net.ls.step(net.msg(1, 1, abi.LEADER_HEARTBEAT), None)
    out = net.ls.last_out
    out = out[out["peer"] % COPIES == 0]
    assert len(out) == 2 and np.all(out["type"] == abi.HEARTBEAT)
    assert np.all(out["log_index"] == 0) and np.all(out["log_term"] == 0) and np.all(out["n_entries"] == 0)
    want = {1: min(off, 5), 2: min(off, off + 11)}  # slot -> commit
    assert {int(m["slot"]): int(m["commit"]) for m in out} == want
    net.close()


# ---- raft_etcd_test.go:2008-2037 TestRecvMsgLeaderHeartbeat
@pytest.mark.parametrize("be", BACKENDS)
@pytest.mark.parametrize("state,wmsg", [(abi.LEADER, 2), (abi.CANDIDATE, 0), (abi.FOLLOWER, 0)])
def test_recv_msg_leader_heartbeat(be, state, wmsg, request):
    ids = [1, 2, 3]
    peers = node_records(ids, set(ids), COPIES)
    for r in range(3):  # log: TestLogDB{entries: [{1, 0}, {2, 1}]} (marker 1, entry 2 at term 1)
        v = peers[r * COPIES:(r + 1) * COPIES]
        v["term"], v["first_index_m1"], v["last_index"], v["n_runs"] = 1, 1, 2, 2
        v["run_start"][:, 0], v["run_term"][:, 0] = 1, 0
        v["run_start"][:, 1], v["run_term"][:, 1] = 2, 1
        v["committed"], v["applied"] = 1, 1
        v["remotes"]["next"] = 3
    peers["state"][:COPIES] = state
    net = Net(_backend(be, request), ids, copies=COPIES, records=peers)
    net.ls.step(net.msg(1, 1, abi.LEADER_HEARTBEAT), None)
    out = net.ls.last_out
    out = out[out["peer"] % COPIES == 0]
    assert len(out) == wmsg and np.all(out["type"] == abi.HEARTBEAT)
    net.close()


# ---- raft_etcd_test.go:272-291 TestLeaderTransferTimeout
@pytest.mark.parametrize("be", BACKENDS)
def test_leader_transfer_timeout(be, request):
    net = Net(_backend(be, request), [1, 2, 3], copies=COPIES)
    _election(net, 1)
    net.isolate(3)
    net.send(net.msg(3, 1, abi.LEADER_TRANSFER, hint=3))
    assert np.all(net.all_copies(1)["leader_transfer_target"] == 3)
    net.tick(1, int(net.state(1)["heartbeat_timeout"]))
    assert np.all(net.all_copies(1)["leader_transfer_target"] == 3)
    net.tick(1, int(net.state(1)["election_timeout"]))
    L = net.all_copies(1)  # checkLeaderTransferState(t, lead, leader, 1)
    assert np.all(L["state"] == abi.LEADER) and np.all(L["leader_id"] == 1)
    assert np.all(L["leader_transfer_target"] == 0)
    net.close()


def _ctx(v):  # readindex_test.go:23-28 getTestSystemCtx
    return v, v + 1


# ---- readindex_test.go:125-162 TestReadIndexLeaderCanBeConfirmed
@pytest.mark.parametrize("be", BACKENDS)
def test_read_index_leader_can_be_confirmed(be, request):
    """The queue of the reference test (requests from nodes 1, 3, 2 at indexes
    3, 4, 5; quorum 3 of 5 voters, leader node 4): the first ack of ctx does not
    confirm, the second releases the first two requests, each answered with
    index 4 (the confirmed request's index) to its requester and the ack's
    context; one request stays queued."""
    ids = [1, 2, 3, 4, 5]
    peers = node_records(ids, set(ids), COPIES)
    for r in range(5):
        v = peers[r * COPIES:(r + 1) * COPIES]
        v["term"], v["committed"], v["applied"], v["last_index"], v["leader_id"] = 2, 5, 5, 5, 4
        v["n_runs"] = 2
        v["run_start"][:, 1], v["run_term"][:, 1] = 1, 2
        v["remotes"]["next"] = 6
    L = peers[3 * COPIES:4 * COPIES]
    L["state"], L["vote"] = abi.LEADER, 4
    L["remotes"]["match"], L["remotes"]["state"] = 5, abi.REPLICATE_ST
    ctx, ctx2, ctx3 = _ctx(10001), _ctx(10002), _ctx(10003)
    ri = L["read_index"]
    for q, (idx, c, frm) in enumerate([(3, ctx2, 1), (4, ctx, 3), (5, ctx3, 2)]):
        ri["index"][:, q], ri["ctx_low"][:, q], ri["ctx_high"][:, q] = idx, c[0], c[1]
        ri["from_slot"][:, q] = frm - 1
    L["read_index_count"] = 3
    net = Net(_backend(be, request), ids, copies=COPIES, records=peers)
    ack = lambda frm: net.msg(frm, 4, abi.HEARTBEAT_RESP, term=2, hint=ctx[0], hint_high=ctx[1])
    net.ls.step(ack(1), None)
    assert np.all(net.all_copies(4)["read_index_count"] == 3)  # confirm(ctx, 1, 3) == nil
    net.ls.step(ack(3), None)
    out = net.ls.last_out
    out = out[(out["peer"] % COPIES == 0) & (out["type"] == abi.READ_INDEX_RESP)]
    got = sorted((int(m["slot"]) + 1, int(m["log_index"]), int(m["hint"]), int(m["hint_high"])) for m in out)
    assert got == [(1, 4, ctx[0], ctx[1]), (3, 4, ctx[0], ctx[1])]
    L = net.all_copies(4)
    assert np.all(L["read_index_count"] == 1) and np.all(L["read_index"]["ctx_low"][:, 0] == ctx3[0])
    net.close()


# ---- raft_test.go:343-420 TestObserverCanReadIndexQuorum1 / Quorum2
@pytest.mark.parametrize("be", BACKENDS)
@pytest.mark.parametrize("voters", [[1], [1, 2]])
def test_observer_can_read_index(be, voters, request):
    ids = [1, 2] if voters == [1] else [1, 2, 3]
    obs = ids[-1]
    net = Net(_backend(be, request), ids, voters=voters, copies=COPIES)
    _election(net, 1)
    assert np.all(net.all_copies(1)["state"] == abi.LEADER)
    for _ in range(int(net.state(1)["randomized_election_timeout"]) + 1):
        net.tick(1)
        net.send(net.msg(1, 1, abi.NOOP))
    assert np.all(net.all_copies(obs)["state"] == abi.OBSERVER)
    committed = _committed(net, 1)
    proposer = 2
    for _ in range(10):
        _propose(net, proposer, proposer)
    assert _committed(net, 1) == committed + 10
    net.send(net.msg(obs, obs, abi.READ_INDEX, hint=12345))
    assert net.ready.get(obs) == [(_committed(net, 1), 12345, 0)], net.ready
    net.close()


# ---- raft_test.go:2057-2081 TestLeaderReadIndexOnSingleNodeCluster
@pytest.mark.parametrize("be", BACKENDS)
def test_leader_read_index_single_node(be, request):
    net = Net(_backend(be, request), [1], copies=COPIES, election=5)
    _election(net, 1)
    n0 = len(net.sent)
    net.local({1: {"read_index": 1, "read_ctx_low": 101, "read_ctx_high": 1002}})
    assert sum(len(s) for s in net.sent[n0:]) == 0  # no message sent
    assert net.ready.get(1) == [(_committed(net, 1), 101, 1002)]
    assert np.all(net.all_copies(1)["read_index_count"] == 0)
    net.close()


# ---- raft_test.go:2083-2102 TestLeaderIgnoregReadIndexWhenClusterCommittedIsUnknown
#      raft_test.go:2104-2141 TestHandleLeaderReadIndex
@pytest.mark.parametrize("be", BACKENDS)
@pytest.mark.parametrize("known", [False, True])
def test_leader_read_index_committed_at_term(be, known, request):
    peers = fresh_leader([1, 2, 3], [1, 2, 3], election=5)
    if known:  # r.remotes[2].tryUpdate(lastIndex); r.tryCommit()
        L = peers[:COPIES]
        L["remotes"]["match"][:, 1], L["remotes"]["next"][:, 1] = 1, 2
        L["committed"] = 1
    net = Net(_backend(be, request), [1, 2, 3], copies=COPIES, records=peers)
    net.ls.step(None, net.locals_({1: {"read_index": 1, "read_ctx_low": 101, "read_ctx_high": 1002}}))
    out = net.ls.last_out
    out = out[out["peer"] % COPIES == 0]
    L = net.all_copies(1)
    if known:
        hb = out[(out["type"] == abi.HEARTBEAT) & (out["hint"] == 101) & (out["hint_high"] == 1002)]
        assert sorted(int(s) + 1 for s in hb["slot"]) == [2, 3]
        assert np.all(L["read_index_count"] == 1)
    else:
        assert len(out) == 0 and np.all(L["read_index_count"] == 0)
    assert not net.ls.last_ready
    net.close()


# ---- BASELINE.json configs[0]: 1 group x 3 replicas, election, 1,000 16-byte
#      proposals one per send, committed/lastIndex traced per node after every send
@pytest.mark.parametrize("be", BACKENDS)
def test_config1_trace(be, request):
    n_props = 1000  # BASELINE config 1 / SURVEY.md §8d: 1,000 16-B proposals on every backend
    net = Net(_backend(be, request), [1, 2, 3], copies=1, payload=16)
    _election(net, 1)
    assert _committed(net, 1) == 1
    for k in range(n_props):
        _propose(net, 1, 1)
        for nid in (1, 2, 3):  # TestLogReplication's expectation after each send
            s = net.state(nid)
            assert int(s["committed"]) == k + 2 and int(s["last_index"]) == k + 2, (k, nid)
    net.close()
