"""SURVEY.md §8f-4 on the device: the in-memory log's persistence marks
(inMemory.savedTo / markerIndex, entryLog.applied) kept in HBM beside the
term-run window, entriesToSave in every result record, and entryLog.commitUpdate
as gr_commit_update.

Known answers transcribed from the reference's tests, each also run by the
oracle (reference table == oracle == engine):
- TestInMemEntriesToSaveReturnNotStabledEntries (inmemory_test.go:349-381)
- TestInMemSaveLogToUpdatesStableTo (inmemory_test.go:383-409)
- TestInMemMergeSetStableTo (inmemory_test.go:426-472), cases 1-2: merge is
  reached through a Replicate whose first conflicting entry is where the table
  merges (the step path calls merge from the conflict index, logentry.go:281-303);
  case 3 merges at an index whose entry matches, which tryAppend never does.
- TestLogCommitUpdateSetsApplied / PanicWhenApplyTwice /
  PanicWhenApplyingNotCommitEntry (logentry_test.go:559-600)
plus randomized parity: leader churn with truncations and partial persistence
acknowledgements, every pass, every peer (marks and result fields).
"""
import numpy as np
import pytest

from dragonboat_amd import abi, populations as P
from oracle.pyoracle import OraclePopulation, hostlane_commit_update, hostlane_step
import parity
import simulate as SIM
from test_golden import _peer, _replicate

BACKENDS = [pytest.param("cpu", id="hostlane"), pytest.param("gpu", id="gpu", marks=pytest.mark.gpu)]


def _need(be, request):
    request.getfixturevalue("gpu" if be == "gpu" else "built")


class _One:
    """One single-peer record driven through the engine (hostlane or GPU) and the oracle."""

    def __init__(self, be, peer, S=3):
        self.be, self.S, self.peer = be, S, peer.copy()
        self.pop = OraclePopulation(peer, S)
        if be == "gpu":
            from dragonboat_amd.engine import Engine
            self.eng = Engine(1, S)
            self.eng.load(peer)

    def step(self, msgs=None, loc=None):
        msgs = np.zeros(0, abi.MESSAGE) if msgs is None else msgs
        loc = np.zeros(0, abi.LOCAL) if loc is None else loc
        if self.be == "gpu":
            out, res = self.eng.step(msgs, loc)
            st = self.eng.sync(1)
        else:
            st, out, res = hostlane_step(self.peer, msgs, loc, self.S)
        self.peer = st
        o = self.pop.step(msgs, loc)
        lim = parity.limits_from(res, 1)
        assert not parity.compare_states(st, o["mid"], self.S)
        assert not parity.compare_msgs(out, parity.prefix_msgs(o, lim))
        assert not parity.compare_results(res, o["results"])
        return st, out, res

    def commit_update(self, uc):
        uc = np.asarray(uc, abi.UPDATE_COMMIT)
        if self.be == "gpu":
            rc, st = self.eng.commit_update(np.zeros(1, np.uint32), uc)
            self.peer = self.eng.sync(1)
        else:
            rc, st = hostlane_commit_update(self.peer, np.zeros(1, np.uint32), uc, self.S)
        orc, ost = self.pop.commit_update(np.zeros(1, np.uint32), uc)
        assert list(st) == list(ost) and (rc == 0) == (orc == 0), (rc, st, orc, ost)
        assert not parity.compare_states(self.peer, self.pop.export(), self.S)
        return int(st[0])

    def close(self):
        if self.be == "gpu":
            self.eng.close()


def _inmem_peer(saved_to, marker=5, last=7, committed=4, log_applied=4):
    """A follower at term 7 whose log is 1..last, entries 5, 6, 7 at terms 5, 6, 7
    (the tables' inMemory; 1..4 at term 5 so the log fits the K = 4 window), in
    memory from `marker`."""
    ents = [(i, 5) for i in range(1, 5)] + [(i, i) for i in range(5, last + 1)]
    p = _peer(3, 3, abi.FOLLOWER, 7, ents, committed)
    p[0]["marker_index"] = marker
    p[0]["saved_to"] = saved_to
    p[0]["log_applied"] = log_applied
    return p


def _qtick():
    loc = np.zeros(1, abi.LOCAL)
    loc["quiesced_ticks"] = 1
    return loc


@pytest.mark.parametrize("be", BACKENDS)
def test_entries_to_save_table(be, request):
    """TestInMemEntriesToSaveReturnNotStabledEntries: savedTo 4 -> [5, 7], 5 -> [6, 7],
    7 -> nothing, 8 -> nothing (gr_peer_result.save_from, 0 = nothing)."""
    _need(be, request)
    for saved, want in [(4, 5), (5, 6), (7, 0), (8, 0)]:
        one = _One(be, _inmem_peer(saved))
        _, _, res = one.step(loc=_qtick())
        assert int(res[0]["save_from"]) == want, (saved, res[0]["save_from"])
        assert int(res[0]["last_index"]) == 7
        one.close()


@pytest.mark.parametrize("be", BACKENDS)
def test_saved_log_to_table(be, request):
    """TestInMemSaveLogToUpdatesStableTo: (index, term) -> savedTo from 4:
    (4, 1) -> 4 (below the marker), (8, 1) -> 4 (past the last entry), (6, 7) -> 4
    (term mismatch), (6, 6) -> 6."""
    _need(be, request)
    for idx, term, want in [(4, 1, 4), (8, 1, 4), (6, 7, 4), (6, 6, 6)]:
        one = _One(be, _inmem_peer(4))
        uc = np.zeros(1, abi.UPDATE_COMMIT)
        uc["stable_log_to"], uc["stable_log_term"] = idx, term
        assert one.commit_update(uc) == 0
        assert int(one.peer[0]["saved_to"]) == want
        one.close()


@pytest.mark.parametrize("be", BACKENDS)
def test_commit_update_applied_table(be, request):
    """TestLogCommitUpdateSetsApplied (committed 10, AppliedTo 5 -> applied 5) and the
    two panics (applied 6: AppliedTo 5 and AppliedTo 12) as status 1, slot untouched;
    appliedLogTo moves markerIndex to AppliedTo inside the in-memory entries."""
    _need(be, request)
    ents = [(i, 1) for i in range(1, 13)]
    for applied, to, want_status in [(0, 5, 0), (6, 5, 1), (6, 12, 1), (6, 10, 0)]:
        p = _peer(3, 3, abi.FOLLOWER, 7, ents, 10)
        p[0]["marker_index"], p[0]["saved_to"], p[0]["log_applied"] = 3, 12, applied
        one = _One(be, p)
        uc = np.zeros(1, abi.UPDATE_COMMIT)
        uc["applied_to"] = to
        assert one.commit_update(uc) == want_status
        if want_status == 0:
            assert int(one.peer[0]["log_applied"]) == to
            assert int(one.peer[0]["marker_index"]) == to  # inMemory.appliedLogTo
        else:
            assert int(one.peer[0]["log_applied"]) == applied and int(one.peer[0]["marker_index"]) == 3
        one.close()


@pytest.mark.parametrize("be", BACKENDS)
def test_merge_sets_saved_to(be, request):
    """TestInMemMergeSetStableTo cases 1-2 through handleReplicateMessage: a
    truncating merge keeps savedTo = min(savedTo, first - 1); a merge at or below
    markerIndex replaces the in-memory log (markerIndex = first, savedTo = first - 1)."""
    _need(be, request)
    # case 1: marker 6, entries 6(6) 7(7), savedTo 5; merge [7 at term 8] -> savedTo 5
    ents = [(i, 1) for i in range(1, 6)] + [(6, 6), (7, 7)]
    p = _peer(3, 3, abi.FOLLOWER, 8, ents, 5)
    p[0]["marker_index"], p[0]["saved_to"], p[0]["log_applied"] = 6, 5, 5
    one = _One(be, p)
    st, _, res = one.step(_replicate(8, 6, 6, 5, [(7, 8)]))
    assert int(st[0]["saved_to"]) == 5 and int(res[0]["save_from"]) == 6
    one.close()
    # case 2: marker 5, entries 5..10, savedTo 4; conflict at 7 -> savedTo 4 (terms
    # 5, 5, 6, 6, 7... instead of 5..10 so the log fits the K = 4 window)
    ents = [(i, 5) for i in range(1, 5)] + [(5, 5), (6, 6)] + [(i, 7) for i in range(7, 11)]
    p = _peer(3, 3, abi.FOLLOWER, 10, ents, 4)
    p[0]["marker_index"], p[0]["saved_to"], p[0]["log_applied"] = 5, 4, 4
    one = _One(be, p)
    st, _, res = one.step(_replicate(10, 6, 6, 4, [(7, 10)]))
    assert int(st[0]["saved_to"]) == 4 and int(st[0]["last_index"]) == 7 and int(res[0]["save_from"]) == 5
    one.close()
    # replace-all: marker 6, savedTo 7 (entries 6, 7 persisted), conflict at 6 -> marker 6, savedTo 5
    ents = [(i, 1) for i in range(1, 6)] + [(6, 6), (7, 6)]
    p = _peer(3, 3, abi.FOLLOWER, 9, ents, 5)
    p[0]["marker_index"], p[0]["saved_to"], p[0]["log_applied"] = 6, 7, 5
    one = _One(be, p)
    st, _, res = one.step(_replicate(9, 5, 1, 5, [(6, 9)]))
    assert int(st[0]["marker_index"]) == 6 and int(st[0]["saved_to"]) == 5 and int(res[0]["save_from"]) == 6
    one.close()


@pytest.mark.parametrize("be", BACKENDS)
def test_persistence_parity_under_churn(be, request):
    """Leader churn (BASELINE config 5's generator: truncations of diverged
    suffixes) with the host acknowledging persistence and apply (gr_commit_update
    + gr_notify_applied) only every third pass: marks, entriesToSave and the
    Update fields equal the oracle's on every peer after every pass."""
    _need(be, request)
    G, R = 400, 3
    backend = SIM.GpuBackend if be == "gpu" else SIM.HostlaneBackend
    peers = P.make_groups(G, R, seed=55)
    topo = P.Topology(G, R)
    rng = np.random.default_rng(55)
    ls = SIM.Lockstep(backend, peers, R)
    msgs = np.zeros(0, abi.MESSAGE)
    saves = 0
    try:
        for k in range(12):
            cur = ls.export()
            ch = P.inject_leader_change(cur, topo, 0.1, rng)
            if len(ch):
                ls.reload(ch, cur[ch])
            loc = P.propose_locals(R * G, P.current_leaders(ls.export(), topo), pass_index=k)
            out, res = ls.step(msgs, loc)
            saves += int(np.count_nonzero(res["save_from"]))
            msgs = topo.route_messages(out)
            if k % 3 == 2:
                ls.apply_all()
    finally:
        ls.close()
    assert saves > 0
