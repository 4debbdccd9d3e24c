"""The reference's own golden tables (tests/golden/raft_tables.json, transcribed by
tests/golden/make_golden.py) driven through the engine's C-ABI record formats:
on the CPU through the test-only host build of the lane code, on the GPU
(-m gpu) through libgpuraft.so. Each case is also run by the oracle, so every
check is three-way: reference table == oracle == engine.

Mapping of each table onto one engine pass (one group, node 1 in slot 0):
- TestCommit (raft_etcd_test.go:1106-1158): a leader at smTerm whose remotes
  have the table's match values (setRemote: state Retry, next = match + 1). The
  reference calls tryCommit directly; here one ReplicateResp from slot 0 raises
  that slot's match from m-1 to m, which runs the same tryCommit.
- TestLogMaybeAppend (logentry_etcd_test.go:172-297): a follower with the table's
  log and committed index receives Replicate{LogIndex, LogTerm, Commit, Entries}
  (handleReplicateMessage, raft.go:953-976, calls matchTerm/tryAppend/commitTo).
  LogIndex < committed answers the committed index before matchTerm
  (raft.go:958-961); those cases (incl. the table's tryAppend panic case, whose
  LogIndex 0 is below committed 1) check that answer and the unchanged commit.
- TestFindConflict (logentry_etcd_test.go:40-72): a follower receives the table's
  entries in a Replicate whose (LogIndex, LogTerm) precede them; the conflict
  index is the first index tryAppend appends (gr_peer_result.append_from).
  Entry lists spanning more than two term runs do not fit one gr_message (the
  host keeps such messages); those cases are checked by the oracle KATs only.
"""
import json
import os

import numpy as np
import pytest

from dragonboat_amd import abi
from oracle.pyoracle import OraclePopulation, hostlane_step
import parity

TABLES = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "raft_tables.json")))


def _slots(n):
    return 1 if n <= 1 else 3 if n <= 3 else 5


def _runs(entries):
    """Term-run window of a log [1..n] over a marker at index 0 with term 0."""
    runs = [(0, 0)]
    for idx, t in entries:
        if runs[-1][1] != t:
            runs.append((idx, t))
    return runs


def _peer(S, voters, state, term, entries, committed):
    p = np.zeros(1, abi.PEER)
    g = p[0]
    g["term"] = term
    g["committed"] = committed
    g["applied"] = committed
    g["last_index"] = entries[-1][0] if entries else 0
    g["first_index_m1"] = 0
    g["node_id"] = 1
    g["leader_id"] = 1 if state == abi.LEADER else 2
    g["election_timeout"] = 10
    g["heartbeat_timeout"] = 1
    g["randomized_election_timeout"] = 10
    g["entry_size_ub"] = 144
    runs = _runs(entries)
    assert len(runs) <= abi.GR_K
    g["n_runs"] = len(runs)
    for k, (s, t) in enumerate(runs):
        g["run_start"][k] = s
        g["run_term"][k] = t
    for j in range(abi.GR_SMAX):
        g["remote_id"][j] = j + 1
        if j < voters:
            g["remotes"][j]["kind"] = abi.SLOT_VOTER
            g["remotes"][j]["next"] = g["last_index"] + 1
            g["remotes"][j]["state"] = abi.RETRY
    g["state"] = state
    g["self_slot"] = 0
    return p


def _replicate(term, log_index, log_term, commit, ents, slot=1):
    m = np.zeros(1, abi.MESSAGE)
    m["peer"] = 0
    m["type"] = abi.REPLICATE
    m["slot"] = slot
    m["term"] = term
    m["log_index"] = log_index
    m["log_term"] = log_term
    m["commit"] = commit
    m["n_entries"] = len(ents)
    if ents:
        terms = [t for _, t in ents]
        cuts = [k for k in range(1, len(terms)) if terms[k] != terms[k - 1]]
        if len(cuts) > 1:
            return None  # more than two runs: not one gr_message
        m["n_runs"] = 1 + len(cuts)
        m["run_term"][0, 0] = terms[0]
        if cuts:
            m["run2_offset"] = cuts[0]
            m["run_term"][0, 1] = terms[cuts[0]]
    return m


def _run_cpu(peer, msgs, S):
    st, out, res = hostlane_step(peer, msgs, None, S)
    return st, out, res


def _run_gpu(peer, msgs, S):
    from dragonboat_amd.engine import Engine
    eng = Engine(1, S)
    eng.load(peer)
    out, res = eng.step(msgs, np.zeros(0, abi.LOCAL))
    st = eng.sync(1)
    eng.close()
    return st, out, res


def _oracle(peer, msgs, S):
    pop = OraclePopulation(peer, S)
    o = pop.step(msgs, np.zeros(0, abi.LOCAL))
    return o


def _check_against_oracle(peer, msgs, S, st, out, res):
    o = _oracle(peer, msgs, S)
    lim = parity.limits_from(res, 1)
    assert not parity.compare_states(st, o["mid"], S)
    assert not parity.compare_msgs(out, parity.prefix_msgs(o, lim))
    assert not parity.compare_results(res, o["results"])


def _commit_case(c, run):
    matches, logs, term, want = c["matches"], c["logs"], c["term"], c["want_committed"]
    S = _slots(len(matches))
    peer = _peer(S, len(matches), abi.LEADER, term, logs, 0)
    for j, m in enumerate(matches):
        peer[0]["remotes"][j]["match"] = m - 1 if j == 0 else m
        peer[0]["remotes"][j]["next"] = m + 1
    resp = np.zeros(1, abi.MESSAGE)
    resp["type"] = abi.REPLICATE_RESP
    resp["slot"] = 0
    resp["term"] = term
    resp["log_index"] = matches[0]
    st, out, res = run(peer, resp, S)
    assert int(st[0]["committed"]) == want
    _check_against_oracle(peer, resp, S, st, out, res)


def _maybe_append_case(c, run, prev, commit0):
    S = 3
    term = 5
    peer = _peer(S, 3, abi.FOLLOWER, term, prev, commit0)
    m = _replicate(term, c["index"], c["log_term"], c["committed"], c["ents"])
    st, out, res = run(peer, m, S)
    resp = out[out["type"] == abi.REPLICATE_RESP]
    if c["index"] < commit0:
        # raft.go:958-961 answers the committed index before matchTerm/tryAppend, so the
        # entryLog-level expectations (incl. the tryAppend panic case) do not apply
        assert len(resp) == 1 and not resp[0]["reject"] and int(resp[0]["log_index"]) == commit0
        assert int(st[0]["committed"]) == commit0
    elif c["want_panic"]:
        assert int(res[0]["escalation"]) == abi.ESC_NAMES.index("panic")
        return
    else:
        assert int(st[0]["committed"]) == c["want_commit"]
        assert len(resp) == 1
        assert bool(resp[0]["reject"]) == (not c["want_append"])
        if c["want_append"]:
            assert int(resp[0]["log_index"]) == c["want_lasti"]
            if c["ents"]:
                assert int(st[0]["last_index"]) == c["want_lasti"]
    _check_against_oracle(peer, m, S, st, out, res)


def _term_at(prev, idx):
    return dict((i, t) for i, t in prev).get(idx, 0)


def _find_conflict_case(c, run, prev):
    S = 3
    term = 5
    ents = c["ents"]
    li = ents[0][0] - 1 if ents else prev[-1][0]
    m = _replicate(term, li, _term_at(prev, li), 0, ents)
    if m is None:
        pytest.skip("more than two term runs in one message (oracle KAT only)")
    peer = _peer(S, 3, abi.FOLLOWER, term, prev, 0)
    st, out, res = run(peer, m, S)
    got = int(res[0]["append_from"]) if len(res) else 0
    assert got == c["want_conflict"]
    _check_against_oracle(peer, m, S, st, out, res)


T = TABLES


@pytest.mark.parametrize("k", range(len(T["TestCommit"]["cases"])))
def test_commit_table_cpu(built, k):
    _commit_case(T["TestCommit"]["cases"][k], _run_cpu)


@pytest.mark.parametrize("k", range(len(T["TestLogMaybeAppend"]["cases"])))
def test_log_maybe_append_table_cpu(built, k):
    t = T["TestLogMaybeAppend"]
    _maybe_append_case(t["cases"][k], _run_cpu, t["previous"], t["committed"])


@pytest.mark.parametrize("k", range(len(T["TestFindConflict"]["cases"])))
def test_find_conflict_table_cpu(built, k):
    t = T["TestFindConflict"]
    _find_conflict_case(t["cases"][k], _run_cpu, t["previous"])


@pytest.mark.gpu
def test_golden_tables_gpu(gpu):
    """Every representable golden case through libgpuraft.so on the GPU."""
    t = T["TestLogMaybeAppend"]
    for c in T["TestCommit"]["cases"]:
        _commit_case(c, _run_gpu)
    for c in t["cases"]:
        _maybe_append_case(c, _run_gpu, t["previous"], t["committed"])
    f = T["TestFindConflict"]
    for c in f["cases"]:
        ents = c["ents"]
        li = ents[0][0] - 1 if ents else f["previous"][-1][0]
        if _replicate(5, li, 0, 0, ents) is None:
            continue
        _find_conflict_case(c, _run_gpu, f["previous"])
