// kat_tests.cpp — TEST INFRASTRUCTURE: pins the oracle against the known-answer
// tests of the reference. Each test names the Go test it
// restates (file:line); the tables are the reference's data, the checking
// code is ours. Build: oracle/Makefile -> oracle/_build/kat_tests.
#include "oracle_testkit.hpp"

#include <algorithm>
#include <cstring>

using namespace oracle;

// ---------------------------------------------------------------- commit (kernel 1)

// raft_etcd_test.go:1106-1158 TestCommit
KAT(TestCommit) {
  struct T {
    std::vector<u64> matches;
    std::vector<Entry> logs;
    u64 smTerm, w;
  };
  std::vector<T> tests = {
      {{1}, E({{1, 1}}), 1, 1},
      {{1}, E({{1, 1}}), 2, 0},
      {{2}, E({{1, 1}, {2, 2}}), 2, 2},
      {{1}, E({{1, 2}}), 2, 1},
      {{2, 1, 1}, E({{1, 1}, {2, 2}}), 1, 1},
      {{2, 1, 1}, E({{1, 1}, {2, 1}}), 2, 0},
      {{2, 1, 2}, E({{1, 1}, {2, 2}}), 2, 2},
      {{2, 1, 2}, E({{1, 1}, {2, 1}}), 2, 0},
      {{2, 1, 1, 1}, E({{1, 1}, {2, 2}}), 1, 1},
      {{2, 1, 1, 1}, E({{1, 1}, {2, 1}}), 2, 0},
      {{2, 1, 1, 2}, E({{1, 1}, {2, 2}}), 1, 1},
      {{2, 1, 1, 2}, E({{1, 1}, {2, 1}}), 2, 0},
      {{2, 1, 2, 2}, E({{1, 1}, {2, 2}}), 2, 2},
      {{2, 1, 2, 2}, E({{1, 1}, {2, 1}}), 2, 0},
  };
  for (auto& tt : tests) {
    TestLogDB storage;
    storage.Append(tt.logs);
    storage.state = State{tt.smTerm, 0, 0};
    auto sm = newTestRaft(1, {1}, 5, 1, &storage);
    for (size_t j = 0; j < tt.matches.size(); j++)
      sm->setRemote(j + 1, tt.matches[j], tt.matches[j] + 1);
    sm->tryCommit();
    EXPECT_EQ(sm->log->committed, tt.w);
  }
}

// raft_test.go:1444-1466 TestUnrolledBubbleSortMatchValue
KAT(TestUnrolledBubbleSortMatchValue) {
  std::vector<std::vector<u64>> tests = {{1, 1, 1}, {1, 1, 2}, {1, 2, 2}, {2, 3, 1}, {3, 2, 1}, {3, 3, 1}};
  for (auto v : tests) {
    auto sm = newTestRaft(1, {1}, 5, 1);
    sm->matched = v;
    sm->sortMatchValues();
    std::sort(v.begin(), v.end());
    EXPECT(sm->matched == v);
  }
}

// raft_test.go:1002-1015 TestQuorumValue, :1017-1026 TestIsSingleNodeQuorum
KAT(TestQuorumValue) {
  EXPECT_EQ(newTestRaft(1, {1}, 5, 1)->quorum(), 1);
  EXPECT_EQ(newTestRaft(1, {1, 2}, 5, 1)->quorum(), 2);
  EXPECT_EQ(newTestRaft(1, {1, 2, 3, 4, 5}, 5, 1)->quorum(), 3);
  EXPECT(newTestRaft(1, {1}, 5, 1)->isSingleNodeQuorum());
  EXPECT(!newTestRaft(1, {1, 2, 3}, 5, 1)->isSingleNodeQuorum());
}

// raft_etcd_test.go:1893-1947 TestLeaderAppResp
KAT(TestLeaderAppResp) {
  struct T {
    u64 index;
    bool reject;
    u64 wmatch, wnext;
    size_t wmsgNum;
    u64 windex, wcommitted;
  };
  std::vector<T> tests = {
      {3, true, 0, 3, 0, 0, 0},
      {2, true, 0, 2, 1, 1, 0},
      {2, false, 2, 4, 2, 2, 2},
      {0, false, 0, 3, 0, 0, 0},
  };
  for (auto& tt : tests) {
    auto sm = newTestRaft(1, {1, 2, 3}, 10, 1);
    TestLogDB db;
    db.entries = E({{1, 0}, {2, 1}});
    sm->log.reset(new entryLog(&db, 3));
    sm->becomeCandidate();
    sm->becomeLeader();
    sm->readMessages();
    Message m = Msg(2, 0, ReplicateResp);
    m.LogIndex = tt.index;
    m.Term = sm->term;
    m.Reject = tt.reject;
    m.Hint = tt.index;
    sm->Handle(m);
    auto& p = sm->remotes[2];
    EXPECT_EQ(p.match, tt.wmatch);
    EXPECT_EQ(p.next, tt.wnext);
    auto msgs = sm->readMessages();
    EXPECT_EQ(msgs.size(), tt.wmsgNum);
    for (auto& x : msgs) {
      EXPECT_EQ(x.LogIndex, tt.windex);
      EXPECT_EQ(x.Commit, tt.wcommitted);
    }
  }
}

// raft_etcd_test.go:2039-2069 TestLeaderIncreaseNext
KAT(TestLeaderIncreaseNext) {
  auto previousEnts = E({{1, 1}, {2, 1}, {3, 1}});
  struct T {
    remoteStateType state;
    u64 next, wnext;
  };
  std::vector<T> tests = {{remoteReplicate, 2, 3 + 1 + 1 + 1}, {remoteRetry, 2, 2}};
  for (auto& tt : tests) {
    auto sm = newTestRaft(1, {1, 2}, 10, 1);
    sm->log->append(previousEnts);
    sm->becomeCandidate();
    sm->becomeLeader();
    sm->remotes[2].state = tt.state;
    sm->remotes[2].next = tt.next;
    sm->Handle(PropMsg(1, 1, "somedata"));
    EXPECT_EQ(sm->remotes[2].next, tt.wnext);
  }
}

// raft_etcd_test.go:1348-1420 TestMTReplicateRespWaitReset
KAT(TestMTReplicateRespWaitReset) {
  auto sm = newTestRaft(1, {1, 2, 3}, 5, 1);
  sm->becomeCandidate();
  sm->becomeLeader();
  sm->broadcastReplicateMessage();
  sm->readMessages();
  Message r2 = Msg(2, 0, ReplicateResp);
  r2.LogIndex = 1;
  sm->Handle(r2);
  EXPECT_EQ(sm->log->committed, 1);
  sm->readMessages();
  Message p = Msg(1, 0, Propose);
  p.Entries.push_back(Entry{});
  sm->Handle(p);
  auto msgs = sm->readMessages();
  EXPECT_EQ(msgs.size(), 1);
  if (msgs.size() == 1) {
    EXPECT(msgs[0].Type == Replicate && msgs[0].To == 2);
    EXPECT(msgs[0].Entries.size() == 1 && msgs[0].Entries[0].Index == 2);
  }
  EXPECT(sm->remotes[3].state == remoteWait);
  Message r3 = Msg(3, 0, ReplicateResp);
  r3.LogIndex = 1;
  sm->Handle(r3);
  EXPECT(sm->remotes[3].state == remoteReplicate);
  msgs = sm->readMessages();
  EXPECT_EQ(msgs.size(), 1);
  if (msgs.size() == 1) {
    EXPECT(msgs[0].Type == Replicate && msgs[0].To == 3);
    EXPECT(msgs[0].Entries.size() == 1 && msgs[0].Entries[0].Index == 2);
  }
}

// raft_etcd_test.go:633-690 TestLogReplication
KAT(TestLogReplication) {
  for (int c = 0; c < 2; c++) {
    network tt({network::fresh(), network::fresh(), network::fresh()});
    std::vector<Message> msgs;
    u64 wcommitted;
    if (c == 0) {
      msgs = {PropMsg(1, 1, "somedata")};
      wcommitted = 2;
    } else {
      msgs = {PropMsg(1, 1, "somedata"), Msg(1, 2, Election), PropMsg(1, 2, "somedata")};
      wcommitted = 4;
    }
    tt.send(Msg(1, 1, Election));
    for (auto& m : msgs) tt.send(m);
    for (auto& kv : tt.peers) {
      raft* sm = kv.second.r;
      EXPECT_EQ(sm->log->committed, wcommitted);
      std::vector<Entry> ents;
      for (auto& e : nextEnts(sm, tt.storage[kv.first].get()))
        if (!e.Cmd.empty()) ents.push_back(e);
      size_t k = 0;
      for (auto& m : msgs) {
        if (m.Type != Propose) continue;
        EXPECT(k < ents.size() && ents[k].Cmd == m.Entries[0].Cmd);
        k++;
      }
    }
  }
}

// raft_etcd_test.go:692-705 TestSingleNodeCommit
KAT(TestSingleNodeCommit) {
  network tt({network::fresh()});
  tt.send(Msg(1, 1, Election));
  tt.send(PropMsg(1, 1, "some data"));
  tt.send(PropMsg(1, 1, "some data"));
  EXPECT_EQ(tt.peer(1)->log->committed, 3);
}

// raft_etcd_test.go:707-749 TestCannotCommitWithoutNewTermEntry
KAT(TestCannotCommitWithoutNewTermEntry) {
  network tt({network::fresh(), network::fresh(), network::fresh(), network::fresh(), network::fresh()});
  tt.send(Msg(1, 1, Election));
  tt.cut(1, 3);
  tt.cut(1, 4);
  tt.cut(1, 5);
  tt.send(PropMsg(1, 1, "some data"));
  tt.send(PropMsg(1, 1, "some data"));
  EXPECT_EQ(tt.peer(1)->log->committed, 1);
  tt.recover();
  tt.ignore(Replicate);
  tt.send(Msg(2, 2, Election));
  raft* sm = tt.peer(2);
  EXPECT_EQ(sm->log->committed, 1);
  tt.recover();
  tt.send(Msg(2, 2, LeaderHeartbeat));
  tt.send(PropMsg(2, 2, "some data"));
  EXPECT_EQ(sm->log->committed, 5);
}

// raft_etcd_test.go:751-779 TestCommitWithoutNewTermEntry
KAT(TestCommitWithoutNewTermEntry) {
  network tt({network::fresh(), network::fresh(), network::fresh(), network::fresh(), network::fresh()});
  tt.send(Msg(1, 1, Election));
  tt.cut(1, 3);
  tt.cut(1, 4);
  tt.cut(1, 5);
  tt.send(PropMsg(1, 1, "some data"));
  tt.send(PropMsg(1, 1, "some data"));
  raft* sm = tt.peer(1);
  EXPECT_EQ(sm->log->committed, 1);
  tt.recover();
  tt.send(Msg(2, 2, Election));
  EXPECT_EQ(sm->log->committed, 4);
}

// raft_etcd_test.go:2595-2664 TestCommitAfterRemoveNode (commit after a voter leaves)
KAT(TestCommitAfterRemoveNodeShape) {
  // restated subset: removeNode() recomputes the quorum and commits.
  auto r = newTestRaft(1, {1, 2}, 5, 1);
  r->becomeCandidate();
  r->becomeLeader();
  r->readMessages();
  u64 before = r->log->committed;
  Message p = Msg(1, 0, Propose);
  p.Entries.push_back(Entry{});
  r->Handle(p);
  EXPECT_EQ(r->log->committed, before);
  r->removeNode(2);
  EXPECT_EQ(r->log->committed, r->log->lastIndex());
}

// ---------------------------------------------------------------- log matching (kernel 2)

// logentry_etcd_test.go:40-72 TestFindConflict
KAT(TestFindConflict) {
  auto prev = E({{1, 1}, {2, 2}, {3, 3}});
  struct T {
    std::vector<Entry> ents;
    u64 w;
  };
  std::vector<T> tests = {
      {{}, 0},
      {E({{1, 1}, {2, 2}, {3, 3}}), 0},
      {E({{2, 2}, {3, 3}}), 0},
      {E({{3, 3}}), 0},
      {E({{1, 1}, {2, 2}, {3, 3}, {4, 4}, {5, 4}}), 4},
      {E({{2, 2}, {3, 3}, {4, 4}, {5, 4}}), 4},
      {E({{3, 3}, {4, 4}, {5, 4}}), 4},
      {E({{4, 4}, {5, 4}}), 4},
      {E({{1, 4}, {2, 4}}), 1},
      {E({{2, 1}, {3, 4}, {4, 4}}), 2},
      {E({{3, 1}, {4, 2}, {5, 4}, {6, 4}}), 3},
  };
  for (auto& tt : tests) {
    TestLogDB db;
    entryLog l(&db);
    l.append(prev);
    EXPECT_EQ(l.getConflictIndex(tt.ents), tt.w);
  }
}

// logentry_test.go:379-414 TestLogMatchTerm, :452-485 TestLogGetConflictIndex
KAT(TestLogMatchTermAndConflictIndex) {
  TestLogDB db;
  db.Append(E({{1, 1}, {2, 1}, {3, 2}, {4, 3}}));
  entryLog el(&db);
  el.append(E({{5, 3}, {6, 3}, {7, 4}}));
  struct M {
    u64 index, term;
    bool match;
  };
  std::vector<M> mt = {{1, 1, true}, {1, 2, false}, {4, 4, false}, {4, 3, true},
                       {5, 3, true}, {5, 4, false}, {7, 4, true},  {8, 5, false}};
  for (auto& t : mt) EXPECT_EQ(el.matchTerm(t.index, t.term), t.match);
  struct C {
    std::vector<Entry> ents;
    u64 conflict;
  };
  std::vector<C> ct = {{{}, 0},
                       {E({{1, 2}}), 1},
                       {E({{1, 1}, {2, 1}}), 0},
                       {E({{1, 1}, {2, 2}}), 2},
                       {E({{6, 3}, {7, 4}}), 0},
                       {E({{6, 3}, {7, 5}}), 7},
                       {E({{7, 4}, {8, 4}}), 8}};
  for (auto& t : ct) EXPECT_EQ(el.getConflictIndex(t.ents), t.conflict);
  // logentry_test.go TestLogUpToDate
  struct U {
    u64 index, term;
    bool ok;
  };
  std::vector<U> ut = {{1, 2, false}, {8, 2, false}, {1, 4, false}, {7, 4, true},
                       {8, 4, true},  {8, 5, true},  {2, 5, true}};
  for (auto& t : ut) EXPECT_EQ(el.upToDate(t.index, t.term), t.ok);
}

// logentry_etcd_test.go:105-162 TestAppend
KAT(TestAppend) {
  auto prev = E({{1, 1}, {2, 2}});
  struct T {
    std::vector<Entry> ents;
    u64 windex;
    std::vector<Entry> wents;
    u64 wunstable;
  };
  std::vector<T> tests = {
      {{}, 2, E({{1, 1}, {2, 2}}), 3},
      {E({{3, 2}}), 3, E({{1, 1}, {2, 2}, {3, 2}}), 3},
      {E({{1, 2}}), 1, E({{1, 2}}), 1},
      {E({{2, 3}, {3, 3}}), 3, E({{1, 1}, {2, 3}, {3, 3}}), 2},
  };
  for (auto& tt : tests) {
    TestLogDB storage;
    storage.Append(prev);
    entryLog l(&storage);
    l.append(tt.ents);
    EXPECT_EQ(l.lastIndex(), tt.windex);
    Err e;
    auto g = l.entries(1, noLimit, &e);
    EXPECT(e == Err::None);
    EXPECT(g == tt.wents);
    EXPECT_EQ(l.inmem.markerIndex, tt.wunstable);
  }
}

// logentry_etcd_test.go:172-297 TestLogMaybeAppend
KAT(TestLogMaybeAppend) {
  auto prev = E({{1, 1}, {2, 2}, {3, 3}});
  const u64 li = 3, lt = 3, commit = 1;
  struct T {
    u64 logTerm, index, committed;
    std::vector<Entry> ents;
    u64 wlasti;
    bool wappend;
    u64 wcommit;
    bool wpanic;
  };
  std::vector<T> tests = {
      {lt - 1, li, li, E({{li + 1, 4}}), 0, false, commit, false},
      {lt, li + 1, li, E({{li + 2, 4}}), 0, false, commit, false},
      {lt, li, li, {}, li, true, li, false},
      {lt, li, li + 1, {}, li, true, li, false},
      {lt, li, li - 1, {}, li, true, li - 1, false},
      {lt, li, 0, {}, li, true, commit, false},
      {0, 0, li, {}, 0, true, commit, false},
      {lt, li, li, E({{li + 1, 4}}), li + 1, true, li, false},
      {lt, li, li + 1, E({{li + 1, 4}}), li + 1, true, li + 1, false},
      {lt, li, li + 2, E({{li + 1, 4}}), li + 1, true, li + 1, false},
      {lt, li, li + 2, E({{li + 1, 4}, {li + 2, 4}}), li + 2, true, li + 2, false},
      {lt - 1, li - 1, li, E({{li, 4}}), li, true, li, false},
      {lt - 2, li - 2, li, E({{li - 1, 4}}), li - 1, true, li - 1, false},
      {lt - 3, li - 3, li, E({{li - 2, 4}}), li - 2, true, li - 2, true},
      {lt - 2, li - 2, li, E({{li - 1, 4}, {li, 4}}), li, true, li, false},
  };
  for (auto& tt : tests) {
    TestLogDB db;
    entryLog l(&db);
    l.append(prev);
    l.committed = commit;
    bool panicked = false;
    try {
      u64 glasti = 0;
      bool gappend = false;
      if (l.matchTerm(tt.index, tt.logTerm)) {
        gappend = true;
        l.tryAppend(tt.index, tt.ents);
        glasti = tt.index + tt.ents.size();
        l.commitTo(min_(glasti, tt.committed));
      }
      EXPECT_EQ(glasti, tt.wlasti);
      EXPECT_EQ(gappend, tt.wappend);
      EXPECT_EQ(l.committed, tt.wcommit);
      if (gappend && !tt.ents.empty()) {
        Err e;
        auto g = l.getEntries(l.lastIndex() - tt.ents.size() + 1, l.lastIndex() + 1, noLimit, &e);
        EXPECT(g == tt.ents);
      }
    } catch (const Panic&) {
      panicked = true;
    }
    EXPECT_EQ(panicked, tt.wpanic);
  }
}

// raft_etcd_test.go:1215-1269 TestHandleMTReplicate
KAT(TestHandleMTReplicate) {
  struct T {
    u64 term, logTerm, logIndex, commit;
    std::vector<Entry> ents;
    u64 wIndex, wCommit;
    bool wReject;
  };
  std::vector<T> tests = {
      {2, 3, 2, 3, {}, 2, 0, true},
      {2, 3, 3, 3, {}, 2, 0, true},
      {2, 1, 1, 1, {}, 2, 1, false},
      {2, 0, 0, 1, E({{1, 2}}), 1, 1, false},
      {2, 2, 2, 3, E({{3, 2}, {4, 2}}), 4, 3, false},
      {2, 2, 2, 4, E({{3, 2}}), 3, 3, false},
      {2, 1, 1, 4, E({{2, 2}}), 2, 2, false},
      {1, 1, 1, 3, {}, 2, 1, false},
      {1, 1, 1, 3, E({{2, 2}}), 2, 2, false},
      {2, 2, 2, 3, {}, 2, 2, false},
      {2, 2, 2, 4, {}, 2, 2, false},
  };
  for (auto& tt : tests) {
    TestLogDB storage;
    storage.Append(E({{1, 1}, {2, 2}}));
    auto sm = newTestRaft(1, {1}, 10, 1, &storage);
    sm->becomeFollower(2, NoLeader);
    Message m;
    m.Type = Replicate;
    m.Term = tt.term;
    m.LogTerm = tt.logTerm;
    m.LogIndex = tt.logIndex;
    m.Commit = tt.commit;
    m.Entries = tt.ents;
    sm->handleReplicateMessage(m);
    EXPECT_EQ(sm->log->lastIndex(), tt.wIndex);
    EXPECT_EQ(sm->log->committed, tt.wCommit);
    auto out = sm->readMessages();
    EXPECT_EQ(out.size(), 1);
    if (out.size() == 1) EXPECT_EQ(out[0].Reject, tt.wReject);
  }
}

// raft_etcd_paper_test.go:583-620 TestFollowerCheckReplicate (exact response incl. Hint)
KAT(TestFollowerCheckReplicate) {
  auto ents = E({{1, 1}, {2, 2}});
  struct T {
    u64 term, index, windex;
    bool wreject;
    u64 whint;
  };
  std::vector<T> tests = {
      {0, 0, 1, false, 0}, {1, 1, 1, false, 0}, {2, 2, 2, false, 0},
      {1, 2, 2, true, 2},  {3, 3, 3, true, 2},
  };
  for (auto& tt : tests) {
    TestLogDB storage;
    storage.Append(ents);
    auto r = newTestRaft(1, {1, 2, 3}, 10, 1, &storage);
    r->loadState(State{0, 0, 1});
    r->becomeFollower(2, 2);
    Message m = Msg(2, 1, Replicate);
    m.Term = 2;
    m.LogTerm = tt.term;
    m.LogIndex = tt.index;
    r->Handle(m);
    auto msgs = r->readMessages();
    EXPECT_EQ(msgs.size(), 1);
    if (msgs.size() == 1) {
      auto& x = msgs[0];
      EXPECT(x.From == 1 && x.To == 2 && x.Type == ReplicateResp && x.Term == 2);
      EXPECT_EQ(x.LogIndex, tt.windex);
      EXPECT_EQ(x.Reject, tt.wreject);
      EXPECT_EQ(x.Hint, tt.whint);
    }
  }
}

// raft_etcd_paper_test.go:627-674 TestFollowerAppendEntries
KAT(TestFollowerAppendEntries) {
  struct T {
    u64 index, term;
    std::vector<Entry> ents, wents, wunstable;
  };
  std::vector<T> tests = {
      {2, 2, E({{3, 3}}), E({{1, 1}, {2, 2}, {3, 3}}), E({{3, 3}})},
      {1, 1, E({{2, 3}, {3, 4}}), E({{1, 1}, {2, 3}, {3, 4}}), E({{2, 3}, {3, 4}})},
      {0, 0, E({{1, 1}}), E({{1, 1}, {2, 2}}), {}},
      {0, 0, E({{1, 3}}), E({{1, 3}}), E({{1, 3}})},
  };
  for (auto& tt : tests) {
    TestLogDB storage;
    storage.Append(E({{1, 1}, {2, 2}}));
    auto r = newTestRaft(1, {1, 2, 3}, 10, 1, &storage);
    r->becomeFollower(2, 2);
    Message m = Msg(2, 1, Replicate);
    m.Term = 2;
    m.LogTerm = tt.term;
    m.LogIndex = tt.index;
    m.Entries = tt.ents;
    r->Handle(m);
    EXPECT(getAllEntries(*r->log) == tt.wents);
    EXPECT(r->log->entriesToSave() == tt.wunstable);
  }
}

// raft_etcd_paper_test.go:679-752 TestLeaderSyncFollowerLog (figure 7 rollback)
static std::string ltoa(const entryLog& l) {
  std::string s = "committed " + std::to_string(l.committed) + " applied " + std::to_string(l.applied);
  for (auto& e : getAllEntries(l)) s += " (" + std::to_string(e.Index) + "," + std::to_string(e.Term) + ")";
  return s;
}
KAT(TestLeaderSyncFollowerLog) {
  auto T = [](std::initializer_list<u64> terms) {
    std::vector<Entry> v(1);  // leading {} entry as in the reference table
    u64 i = 1;
    for (u64 t : terms) { Entry e; e.Index = i++; e.Term = t; v.push_back(e); }
    return v;
  };
  auto ents = T({1, 1, 1, 4, 4, 5, 5, 6, 6, 6});
  u64 term = 8;
  std::vector<std::vector<Entry>> tests = {
      T({1, 1, 1, 4, 4, 5, 5, 6, 6}),
      T({1, 1, 1, 4}),
      T({1, 1, 1, 4, 4, 5, 5, 6, 6, 6, 6}),
      T({1, 1, 1, 4, 4, 5, 5, 6, 6, 6, 7, 7}),
      T({1, 1, 1, 4, 4, 4, 4}),
      T({1, 1, 1, 2, 2, 2, 3, 3, 3, 3, 3}),
  };
  for (auto& tt : tests) {
    TestLogDB leadStorage;
    leadStorage.Append(ents);
    auto lead = newTestRaft(1, {1, 2, 3}, 10, 1, &leadStorage);
    lead->loadState(State{term, 0, lead->log->lastIndex()});
    TestLogDB followerStorage;
    followerStorage.Append(tt);
    auto follower = newTestRaft(2, {1, 2, 3}, 10, 1, &followerStorage);
    follower->loadState(State{term - 1, 0, 0});
    network n({network::use(lead.get()), network::use(follower.get()), network::hole()});
    n.send(Msg(1, 1, Election));
    Message v = Msg(3, 1, RequestVoteResp);
    v.Term = term + 1;
    n.send(v);
    Message p = Msg(1, 1, Propose);
    p.Entries.push_back(Entry{});
    n.send(p);
    EXPECT(ltoa(*lead->log) == ltoa(*follower->log));
  }
}

// raft_etcd_test.go:1272-1302 TestHandleHeartbeat
KAT(TestHandleHeartbeat) {
  u64 commit = 2;
  struct T {
    u64 mcommit, wCommit;
  };
  std::vector<T> tests = {{commit + 1, commit + 1}, {commit - 1, commit}};
  for (auto& tt : tests) {
    TestLogDB storage;
    storage.Append(E({{1, 1}, {2, 2}, {3, 3}}));
    auto sm = newTestRaft(1, {1, 2}, 5, 1, &storage);
    sm->becomeFollower(2, 2);
    sm->log->commitTo(commit);
    Message m = Msg(2, 1, Heartbeat);
    m.Term = 2;
    m.Commit = tt.mcommit;
    sm->handleHeartbeatMessage(m);
    EXPECT_EQ(sm->log->committed, tt.wCommit);
    auto out = sm->readMessages();
    EXPECT(out.size() == 1 && out[0].Type == HeartbeatResp);
  }
}

// raft_etcd_test.go:1305-1346 TestHandleHeartbeatResp
KAT(TestHandleHeartbeatResp) {
  TestLogDB storage;
  storage.Append(E({{1, 1}, {2, 2}, {3, 3}}));
  auto sm = newTestRaft(1, {1, 2}, 5, 1, &storage);
  sm->becomeCandidate();
  sm->becomeLeader();
  sm->log->commitTo(sm->log->lastIndex());
  sm->Handle(Msg(2, 0, HeartbeatResp));
  auto msgs = sm->readMessages();
  EXPECT(msgs.size() == 1 && msgs[0].Type == Replicate);
  sm->Handle(Msg(2, 0, HeartbeatResp));
  msgs = sm->readMessages();
  EXPECT(msgs.size() == 1 && msgs[0].Type == Replicate);
  Message r = Msg(2, 0, ReplicateResp);
  r.LogIndex = msgs[0].LogIndex + msgs[0].Entries.size();
  sm->Handle(r);
  sm->readMessages();
  sm->Handle(Msg(2, 0, HeartbeatResp));
  EXPECT_EQ(sm->readMessages().size(), 0);
}

// ---------------------------------------------------------------- remote (flow control)

// remote_test.go:192-221 TestRemoteRespondedTo
KAT(TestRemoteRespondedTo) {
  struct T {
    remoteStateType st;
    u64 match, next, si;
    remoteStateType expSt;
    u64 expNext;
  };
  std::vector<T> tests = {{remoteRetry, 10, 12, 0, remoteReplicate, 11},
                          {remoteReplicate, 10, 12, 0, remoteReplicate, 12},
                          {remoteSnapshot, 10, 12, 8, remoteRetry, 11},
                          {remoteSnapshot, 10, 11, 12, remoteSnapshot, 11}};
  for (auto& tt : tests) {
    remote r;
    r.state = tt.st;
    r.match = tt.match;
    r.next = tt.next;
    r.snapshotIndex = tt.si;
    r.respondedTo();
    EXPECT(r.state == tt.expSt);
    EXPECT_EQ(r.next, tt.expNext);
  }
}

// remote_test.go:223-264 TestRemoteTryUpdate
KAT(TestRemoteTryUpdate) {
  const u64 match = 10, next = 20;
  struct T {
    u64 index;
    bool paused;
    u64 expMatch, expNext;
    bool expPaused, expUpdated;
  };
  std::vector<T> tests = {
      {next, false, next, next + 1, false, true},         {next, true, next, next + 1, false, true},
      {next - 2, false, next - 2, next, false, true},     {next - 2, true, next - 2, next, false, true},
      {next - 1, false, next - 1, next, false, true},     {next - 1, true, next - 1, next, false, true},
      {match - 1, false, match, next, false, false},      {match - 1, true, match, next, true, false},
  };
  for (auto& tt : tests) {
    remote r;
    r.match = match;
    r.next = next;
    if (tt.paused) r.retryToWait();
    bool updated = r.tryUpdate(tt.index);
    EXPECT_EQ(updated, tt.expUpdated);
    EXPECT(r.next == tt.expNext && r.match == tt.expMatch);
    if (tt.expPaused) EXPECT(r.state == remoteWait);
  }
}

// remote_test.go:266-321 TestRemoteDecreaseTo{In,Not}ReplicateState
KAT(TestRemoteDecreaseTo) {
  struct A {
    u64 match, next, rejected;
    bool decreased;
    u64 expNext;
  };
  for (auto& tt : std::vector<A>{{10, 15, 9, false, 15}, {10, 15, 10, false, 15}, {10, 15, 12, true, 11}}) {
    remote r;
    r.match = tt.match;
    r.next = tt.next;
    r.state = remoteReplicate;
    EXPECT_EQ(r.decreaseTo(tt.rejected, 100), tt.decreased);
    EXPECT_EQ(r.next, tt.expNext);
  }
  struct B {
    u64 match, next, rejected, last;
    bool decreased;
    u64 expNext;
  };
  for (auto& tt : std::vector<B>{{10, 15, 20, 100, false, 15}, {10, 15, 14, 100, true, 14}, {10, 15, 14, 10, true, 11}}) {
    for (auto st : {remoteRetry, remoteSnapshot}) {
      remote r;
      r.match = tt.match;
      r.next = tt.next;
      r.state = st;
      r.retryToWait();
      EXPECT_EQ(r.decreaseTo(tt.rejected, tt.last), tt.decreased);
      EXPECT_EQ(r.next, tt.expNext);
      if (tt.decreased) EXPECT(r.state != remoteWait);
    }
  }
  // remote_test.go:323-335 TestRemoteTryUpdateCauseResume
  remote r;
  r.next = 5;
  r.retryToWait();
  r.decreaseTo(4, 4);
  EXPECT(r.state != remoteWait);
  r.retryToWait();
  r.tryUpdate(5);
  EXPECT(r.state != remoteWait);
}

// ---------------------------------------------------------------- ReadIndex (kernel 3)

static SystemCtx getTestSystemCtx(u64 v) { return SystemCtx{v, v + 1}; }  // readindex_test.go:23-28

// readindex_test.go:30-40, 55-82, 84-101, 125-162
KAT(TestReadIndexQueue) {
  {
    readIndex r;
    r.addRequest(1, getTestSystemCtx(10001), 1);
    EXPECT_EQ(r.pending.size(), 1);
    r.addRequest(2, getTestSystemCtx(10001), 2);
    EXPECT_EQ(r.pending.size(), 1);
  }
  {
    readIndex r;
    r.addRequest(1, getTestSystemCtx(10001), 1);
    r.addRequest(2, getTestSystemCtx(10002), 2);
    EXPECT(r.hasPendingRequest());
    EXPECT(r.queue.size() == 2 && r.pending.size() == 2);
    auto p = r.pending[getTestSystemCtx(10002)];
    EXPECT(p->index == 2 && p->from == 2 && p->ctx == getTestSystemCtx(10002));
    EXPECT(r.peepCtx() == getTestSystemCtx(10002));
  }
  {
    readIndex r;
    r.addRequest(3, getTestSystemCtx(10001), 1);
    r.addRequest(5, getTestSystemCtx(10002), 3);
    EXPECT_PANIC(r.addRequest(4, getTestSystemCtx(10003), 2));
  }
  {
    readIndex r;
    auto ctx = getTestSystemCtx(10001), ctx2 = getTestSystemCtx(10002), ctx3 = getTestSystemCtx(10003);
    r.addRequest(3, ctx2, 1);
    r.addRequest(4, ctx, 3);
    r.addRequest(5, ctx3, 2);
    auto ris = r.confirm(ctx, 1, 3);
    EXPECT(ris.empty());
    ris = r.confirm(ctx, 3, 3);
    EXPECT_EQ(ris.size(), 2);
    if (ris.size() == 2) {
      EXPECT(ris[1]->index == 4 && ris[1]->from == 3 && ris[1]->ctx == ctx);
      EXPECT(ris[0]->index == 4 && ris[0]->from == 1 && ris[0]->ctx == ctx2);
    }
    EXPECT(r.pending.size() == 1 && r.queue.size() == 1);
  }
}

// raft_test.go:950-971 TestBroadcastHeartbeatMessageWithHint, :984-1000 TestSendHeartbeatMessage
KAT(TestHeartbeatWithHint) {
  SystemCtx ctx{101, 1001};
  auto r = newTestRaft(1, {1, 2, 3}, 5, 1);
  r->becomeCandidate();
  r->becomeLeader();
  r->readMessages();
  r->broadcastHeartbeatMessageWithHint(ctx);
  int count = 0;
  for (auto& m : r->msgs) {
    if (m.Type == Heartbeat) count++;
    EXPECT(m.Hint == ctx.Low && m.HintHigh == ctx.High);
  }
  EXPECT_EQ(count, 2);
  auto r2 = newTestRaft(1, {1, 2}, 5, 1);
  r2->becomeCandidate();
  r2->becomeLeader();
  r2->readMessages();
  r2->remotes[2].match = 100;
  r2->log->committed = 200;
  r2->sendHeartbeatMessage(2, SystemCtx{100, 200}, false);
  EXPECT(r2->msgs.size() == 1 && r2->msgs[0].Commit == 100 && r2->msgs[0].Hint == 100 &&
         r2->msgs[0].HintHigh == 200);
}

// raft_test.go:2057-2141 leader ReadIndex handling
KAT(TestHandleLeaderReadIndex) {
  {  // TestLeaderReadIndexOnSingleNodeCluster
    auto r = newTestRaft(1, {1}, 5, 1);
    r->becomeCandidate();
    r->becomeLeader();
    r->readMessages();
    Message m = Msg(0, 0, ReadIndex);
    m.Hint = 101;
    m.HintHigh = 1002;
    r->handleLeaderReadIndex(m);
    EXPECT_EQ(r->msgs.size(), 0);
    EXPECT_EQ(r->readyToRead.size(), 1);
    EXPECT(r->readyToRead[0].Index == r->log->committed && r->readyToRead[0].ctx.Low == 101 &&
           r->readyToRead[0].ctx.High == 1002);
  }
  {  // TestLeaderIgnoregReadIndexWhenClusterCommittedIsUnknown
    auto r = newTestRaft(1, {1, 2, 3}, 5, 1);
    r->becomeCandidate();
    r->becomeLeader();
    r->readMessages();
    Message m = Msg(0, 0, ReadIndex);
    m.Hint = 101;
    m.HintHigh = 1002;
    r->handleLeaderReadIndex(m);
    EXPECT(r->msgs.empty() && r->readyToRead.empty() && r->readIdx.queue.empty());
  }
  {  // TestLeaderIgnoregReadIndexWhenSelfRemoved
    auto r = newTestRaft(1, {1, 2, 3}, 5, 1);
    r->becomeCandidate();
    r->becomeLeader();
    r->readMessages();
    r->deleteRemote(r->nodeID);
    EXPECT(r->selfRemoved());
    Message m = Msg(0, 0, ReadIndex);
    m.Hint = 101;
    m.HintHigh = 1002;
    r->handleLeaderReadIndex(m);
    EXPECT(r->msgs.empty() && r->readyToRead.empty() && r->readIdx.queue.empty());
  }
  {  // TestHandleLeaderReadIndex
    auto r = newTestRaft(1, {1, 2, 3}, 5, 1);
    r->becomeFollower(1, NoLeader);
    EXPECT(!r->hasCommittedEntryAtCurrentTerm());
    r->becomeCandidate();
    r->becomeLeader();
    r->readMessages();
    EXPECT(!r->hasCommittedEntryAtCurrentTerm());
    r->remotes[2].tryUpdate(r->log->lastIndex());
    EXPECT(r->tryCommit());
    EXPECT(r->hasCommittedEntryAtCurrentTerm());
    Message m = Msg(0, 0, ReadIndex);
    m.Hint = 101;
    m.HintHigh = 1002;
    r->handleLeaderReadIndex(m);
    int count = 0;
    for (auto& x : r->msgs)
      if (x.Type == Heartbeat && (x.To == 2 || x.To == 3) && x.Hint == 101 && x.HintHigh == 1002) count++;
    EXPECT_EQ(count, 2);
    EXPECT(r->readIdx.pending.size() == 1 && r->readIdx.queue.size() == 1);
  }
}

// raft_test.go:343-420 TestObserverCanReadIndexQuorum{1,2}
static std::unique_ptr<raft> newTestObserver(u64 id, std::vector<u64> peers, std::vector<u64> obs,
                                             u64 election, u64 heartbeat, TestLogDB* db) {
  Config cfg = newTestConfig(id, election, heartbeat);
  cfg.IsObserver = true;
  std::unique_ptr<raft> r(new raft(cfg, db));
  if (r->remotes.empty())
    for (u64 p : peers) { remote x; x.next = 1; r->remotes[p] = x; }
  if (r->observers.empty())
    for (u64 p : obs) { remote x; x.next = 1; r->observers[p] = x; }
  raft* rp = r.get();
  r->hasNotAppliedConfigChange = [rp]() { return rp->testOnlyHasConfigChangeToApply(); };
  return r;
}
KAT(TestObserverCanReadIndexQuorum) {
  {
    TestLogDB d1, d2;
    auto p1 = newTestObserver(1, {}, {1, 2}, 10, 1, &d1);
    auto p2 = newTestObserver(2, {}, {1, 2}, 10, 1, &d2);
    p1->addNode(1);
    p2->addNode(1);
    EXPECT(!p1->isObserver());
    EXPECT(p2->isObserver());
    network nt({network::use(p1.get()), network::use(p2.get())});
    EXPECT_EQ(p1->remotes.size(), 1);
    nt.send(Msg(1, 1, Election));
    EXPECT(p1->state == leader);
    for (u64 i = 0; i <= p1->randomizedElectionTimeout; i++) {
      p1->tick();
      nt.send(Msg(1, 1, NoOP));
    }
    EXPECT(p2->isObserver());
    u64 committed = p1->log->committed;
    for (int i = 0; i < 10; i++) nt.send(PropMsg(2, 2, "test-data"));
    EXPECT_EQ(committed + 10, p1->log->committed);
    Message ri = Msg(2, 2, ReadIndex);
    ri.Hint = 12345;
    nt.send(ri);
    EXPECT_EQ(p2->readyToRead.size(), 1);
    if (!p2->readyToRead.empty()) EXPECT_EQ(p2->readyToRead[0].Index, p1->log->committed);
  }
  {
    TestLogDB d1, d2, d3;
    auto p1 = newTestRaftOn(1, {1, 2}, 10, 1, &d1);
    auto p2 = newTestRaftOn(2, {1, 2}, 10, 1, &d2);
    auto p3 = newTestObserver(3, {1, 2}, {3}, 10, 1, &d3);
    p1->addObserver(3);
    p2->addObserver(3);
    network nt({network::use(p1.get()), network::use(p2.get()), network::use(p3.get())});
    nt.send(Msg(1, 1, Election));
    EXPECT(p1->state == leader);
    EXPECT(p2->state == follower);
    EXPECT(p3->isObserver());
    for (u64 i = 0; i <= p1->randomizedElectionTimeout; i++) {
      p1->tick();
      nt.send(Msg(1, 1, NoOP));
    }
    u64 committed = p1->log->committed;
    for (int i = 0; i < 10; i++) nt.send(PropMsg(2, 2, "test-data"));
    EXPECT_EQ(committed + 10, p1->log->committed);
    Message ri = Msg(3, 3, ReadIndex);
    ri.Hint = 12345;
    nt.send(ri);
    EXPECT_EQ(p3->readyToRead.size(), 1);
    if (!p3->readyToRead.empty()) EXPECT_EQ(p3->readyToRead[0].Index, p1->log->committed);
  }
}

// ---------------------------------------------------------------- ticks (kernel 4)

// raft_test.go:574-589 TestFollowerTick
KAT(TestFollowerTick) {
  auto r = newTestRaft(1, {1, 2}, 5, 1);
  r->becomeFollower(10, 2);
  for (int i = 0; i < 9; i++) {
    EXPECT(!r->timeForElection());
    r->tick();
  }
  EXPECT_EQ(r->msgs.size(), 1);
  if (!r->msgs.empty()) EXPECT(r->msgs[0].Type == RequestVote);
}
// The count of ticks before the election in TestFollowerTick depends on the
// randomized timeout; pin it as setRandomizedElectionTimeout does.
KAT(TestFollowerTickPinned) {
  auto r = newTestRaft(1, {1, 2}, 5, 1);
  r->becomeFollower(10, 2);
  r->randomizedElectionTimeout = 7;
  for (int i = 0; i < 6; i++) r->tick();
  EXPECT_EQ(r->msgs.size(), 0);
  r->tick();
  EXPECT_EQ(r->msgs.size(), 1);
  EXPECT_EQ(r->electionTick, 0);
  EXPECT(r->state == candidate);
}

// raft_test.go:591-606 TestLeaderTick
KAT(TestLeaderTick) {
  auto r = newTestRaft(1, {1, 2}, 5, 1);
  r->becomeCandidate();
  r->becomeLeader();
  for (int i = 0; i < 10; i++) r->tick();
  EXPECT_EQ(r->msgs.size(), 10);
  for (auto& m : r->msgs) EXPECT(m.Type == Heartbeat);
}

// raft_test.go:608-622 TestTimeForElection
KAT(TestTimeForElection) {
  auto r = newTestRaft(1, {1}, 5, 1);
  EXPECT(r->randomizedElectionTimeout >= 5 && r->randomizedElectionTimeout <= 10);
  r->electionTick = r->randomizedElectionTimeout - 1;
  EXPECT(!r->timeForElection());
  r->electionTick = r->randomizedElectionTimeout;
  EXPECT(r->timeForElection());
}

// raft_test.go:624-635 TestLeaderChecksQuorumEveryElectionTick
KAT(TestLeaderChecksQuorumEveryElectionTick) {
  auto r = newTestRaft(1, {1, 2}, 5, 1);
  r->becomeCandidate();
  r->becomeLeader();
  r->checkQuorum = true;
  for (int i = 0; i < 5; i++) r->tick();
  EXPECT(r->state != leader);
}

// raft_test.go:637-655 TestQuiescedTick
KAT(TestQuiescedTick) {
  auto r = newTestRaft(1, {1, 2}, 5, 1);
  r->becomeCandidate();
  r->becomeLeader();
  r->readMessages();
  for (int i = 0; i < 200; i++) r->quiescedTick();
  EXPECT_EQ(r->msgs.size(), 0);
  auto f = newTestRaft(1, {1, 2}, 5, 1);
  f->becomeFollower(10, 2);
  for (int i = 0; i < 200; i++) f->quiescedTick();
  EXPECT_EQ(f->msgs.size(), 0);
  EXPECT_EQ(f->electionTick, 200);
}

// raft_etcd_test.go:1602-1635 TestLeaderStepdownWhenQuorum{Active,Lost}
KAT(TestLeaderStepdownWhenQuorum) {
  {
    auto sm = newTestRaft(1, {1, 2, 3}, 5, 1);
    sm->checkQuorum = true;
    sm->becomeCandidate();
    sm->becomeLeader();
    for (u64 i = 0; i < sm->electionTimeout + 1; i++) {
      Message m = Msg(2, 0, HeartbeatResp);
      m.Term = sm->term;
      sm->Handle(m);
      sm->tick();
    }
    EXPECT(sm->state == leader);
  }
  {
    auto sm = newTestRaft(1, {1, 2, 3}, 5, 1);
    sm->checkQuorum = true;
    sm->becomeCandidate();
    sm->becomeLeader();
    for (u64 i = 0; i < sm->electionTimeout + 1; i++) sm->tick();
    EXPECT(sm->state == follower);
  }
}

// raft_test.go:1310-1327 TestHandleLeaderCheckQuorum
KAT(TestHandleLeaderCheckQuorum) {
  auto r = newTestRaft(1, {1, 2}, 5, 1);
  r->becomeCandidate();
  r->becomeLeader();
  r->handleLeaderCheckQuorum(Message{});
  EXPECT(r->state == follower);
  auto r2 = newTestRaft(1, {1, 2}, 5, 1);
  r2->becomeCandidate();
  r2->becomeLeader();
  r2->remotes[1].setActive();
  r2->remotes[2].setActive();
  r2->handleLeaderCheckQuorum(Message{});
  EXPECT(r2->state == leader);
}

// raft_etcd_test.go:1951-2005 TestBcastBeat
KAT(TestBcastBeat) {
  u64 offset = 1000;
  Snapshot s;
  s.Index = offset;
  s.Term = 1;
  s.membership = getTestMembership({1, 2, 3});
  TestLogDB storage;
  storage.ApplySnapshot(s);
  auto sm = newTestRaft(1, {}, 10, 1, &storage);
  sm->term = 1;
  sm->becomeCandidate();
  sm->becomeLeader();
  for (int i = 0; i < 10; i++) {
    std::vector<Entry> es(1);
    es[0].Index = i + 1;
    sm->appendEntries(es);
  }
  sm->remotes[2].match = 5;
  sm->remotes[2].next = 6;
  sm->remotes[3].match = sm->log->lastIndex();
  sm->remotes[3].next = sm->log->lastIndex() + 1;
  sm->readMessages();
  sm->Handle(Msg(0, 0, LeaderHeartbeat));
  auto msgs = sm->readMessages();
  EXPECT_EQ(msgs.size(), 2);
  std::map<u64, u64> want = {{2, min_(sm->log->committed, sm->remotes[2].match)},
                             {3, min_(sm->log->committed, sm->remotes[3].match)}};
  for (auto& m : msgs) {
    EXPECT(m.Type == Heartbeat && m.LogIndex == 0 && m.LogTerm == 0 && m.Entries.empty());
    EXPECT(want.count(m.To) && m.Commit == want[m.To]);
  }
}

// raft_etcd_test.go:2008-2037 TestRecvMsgLeaderHeartbeat
KAT(TestRecvMsgLeaderHeartbeat) {
  struct T {
    RaftState st;
    size_t wMsg;
  };
  for (auto& tt : std::vector<T>{{leader, 2}, {candidate, 0}, {follower, 0}}) {
    auto sm = newTestRaft(1, {1, 2, 3}, 10, 1);
    TestLogDB db;
    db.entries = E({{1, 0}, {2, 1}});
    sm->log.reset(new entryLog(&db, 0));
    sm->term = 1;
    sm->state = tt.st;
    sm->Handle(Msg(1, 1, LeaderHeartbeat));
    auto msgs = sm->readMessages();
    EXPECT_EQ(msgs.size(), tt.wMsg);
    for (auto& m : msgs) EXPECT(m.Type == Heartbeat);
  }
}

// raft_etcd_test.go:272-292 TestLeaderTransferTimeout
KAT(TestLeaderTransferTimeout) {
  network nt({network::fresh(), network::fresh(), network::fresh()});
  nt.send(Msg(1, 1, Election));
  nt.isolate(3);
  raft* lead = nt.peer(1);
  Message lt = Msg(3, 1, LeaderTransfer);
  lt.Hint = 3;
  nt.send(lt);
  EXPECT_EQ(lead->leaderTransferTarget, 3);
  for (u64 i = 0; i < lead->heartbeatTimeout; i++) lead->tick();
  EXPECT_EQ(lead->leaderTransferTarget, 3);
  for (u64 i = 0; i < lead->electionTimeout; i++) lead->tick();
  EXPECT(lead->state == leader && lead->leaderID == 1 && lead->leaderTransferTarget == NoNode);
}

int main(int argc, char** argv) {
  int failedTests = 0;
  for (auto& t : registry()) {
    if (argc > 1 && strcmp(argv[1], t.name) != 0) continue;
    int before = failures();
    try {
      t.fn();
    } catch (const std::exception& e) {
      failures()++;
      fprintf(stderr, "  uncaught exception: %s\n", e.what());
    }
    bool ok = failures() == before;
    if (!ok) failedTests++;
    printf("%s %s\n", ok ? "PASS" : "FAIL", t.name);
  }
  printf("%zu tests, %d failed\n", registry().size(), failedTests);
  return failedTests ? 1 : 0;
}
