// oracle_testkit.hpp — TEST INFRASTRUCTURE: helpers that mirror the fixtures
// of the reference's raft tests, so transcribed known-answer tests read like
// the originals.
//   newTestConfig/newTestRaft/newTestObserver  raft_etcd_test.go:2955-2990
//   network (FIFO send loop, drop/cut/isolate/ignore/recover, blackHole)
//                                              raft_etcd_test.go:2803-2938
//   nextEnts                                   raft_etcd_test.go:97-110
//   getAllEntries                              logentry_etcd_test.go:28-38
#pragma once
#include "raft_oracle.hpp"

#include <cstdio>
#include <map>
#include <memory>
#include <cstring>
#include <set>
#include <string>
#include <vector>

namespace oracle {

inline Config newTestConfig(u64 id, u64 election, u64 heartbeat) {
  Config c;
  c.NodeID = id;
  c.ElectionRTT = election;
  c.HeartbeatRTT = heartbeat;
  return c;
}

// Owns the logdb alongside the raft so tests can keep raw pointers.
struct TestNode {
  std::unique_ptr<TestLogDB> ownedDB;
  std::unique_ptr<raft> r;
  raft* operator->() { return r.get(); }
  raft* get() { return r.get(); }
};

inline std::unique_ptr<raft> newTestRaftOn(u64 id, const std::vector<u64>& peers, u64 election,
                                           u64 heartbeat, ILogDB* logdb) {
  std::unique_ptr<raft> r(new raft(newTestConfig(id, election, heartbeat), logdb));
  if (r->remotes.empty())
    for (u64 p : peers) { remote rm; rm.next = 1; r->remotes[p] = rm; }
  raft* rp = r.get();
  r->hasNotAppliedConfigChange = [rp]() { return rp->testOnlyHasConfigChangeToApply(); };
  return r;
}

inline TestNode newTestRaft(u64 id, const std::vector<u64>& peers, u64 election, u64 heartbeat,
                            TestLogDB* db = nullptr) {
  TestNode n;
  if (!db) { n.ownedDB.reset(new TestLogDB()); db = n.ownedDB.get(); }
  n.r = newTestRaftOn(id, peers, election, heartbeat, db);
  return n;
}

inline Membership getTestMembership(const std::vector<u64>& nodes) {
  Membership m;
  for (u64 n : nodes) m.Addresses[n] = "";
  return m;
}

inline std::vector<Entry> E(std::initializer_list<std::pair<u64, u64>> idxTerm) {
  std::vector<Entry> v;
  for (auto& p : idxTerm) { Entry e; e.Index = p.first; e.Term = p.second; v.push_back(e); }
  return v;
}

inline std::vector<Entry> getAllEntries(const entryLog& l) {
  Err e;
  auto ents = l.entries(l.firstIndex(), noLimit, &e);
  if (e == Err::None) return ents;
  if (e == Err::Compacted) return getAllEntries(l);
  panicf("getAllEntries");
}

inline std::vector<Entry> nextEnts(raft* r, ILogDB* s) {
  s->Append(r->log->entriesToSave());
  UpdateCommit uc;
  uc.StableLogTo = r->log->lastIndex();
  uc.StableLogTerm = r->log->lastTerm();
  r->log->commitUpdate(uc);
  auto ents = r->log->entriesToApply();
  UpdateCommit ac;
  ac.AppliedTo = r->log->committed;
  r->log->commitUpdate(ac);
  return ents;
}

// The in-memory multi-node network of raft_etcd_test.go:2803-2938. Peers are
// either raft instances or black holes. Delivery is a FIFO work queue.
struct network {
  struct Slot {
    raft* r = nullptr;  // nullptr => blackHole
  };
  std::map<u64, Slot> peers;
  std::map<u64, std::unique_ptr<TestLogDB>> storage;
  std::vector<std::unique_ptr<raft>> owned;
  std::map<std::pair<u64, u64>, double> dropm;
  std::set<MessageType> ignorem;
  SplitMix64 rnd{12345};

  // spec: 'n' = new default peer, 'b' = black hole, or an existing raft*.
  struct PeerSpec {
    char kind;
    raft* r;
  };
  static PeerSpec fresh() { return {'n', nullptr}; }
  static PeerSpec hole() { return {'b', nullptr}; }
  static PeerSpec use(raft* r) { return {'r', r}; }

  explicit network(std::vector<PeerSpec> specs, void (*cfgf)(Config*) = nullptr) {
    size_t size = specs.size();
    std::vector<u64> addrs;
    for (size_t i = 0; i < size; i++) addrs.push_back(1 + i);
    for (size_t j = 0; j < size; j++) {
      u64 id = addrs[j];
      auto& sp = specs[j];
      if (sp.kind == 'n') {
        storage[id].reset(new TestLogDB());
        Config cfg = newTestConfig(id, 10, 1);
        if (cfgf) cfgf(&cfg);
        std::unique_ptr<raft> sm(new raft(cfg, storage[id].get()));
        sm->setTestPeers(addrs);
        raft* rp = sm.get();
        sm->hasNotAppliedConfigChange = [rp]() { return rp->testOnlyHasConfigChangeToApply(); };
        peers[id].r = rp;
        owned.push_back(std::move(sm));
      } else if (sp.kind == 'r') {
        raft* v = sp.r;
        std::set<u64> obs;
        for (auto& kv : v->observers) obs.insert(kv.first);
        v->nodeID = id;
        v->remotes.clear();
        v->observers.clear();
        for (size_t i = 0; i < size; i++) {
          if (obs.count(addrs[i])) v->observers[addrs[i]] = remote{};
          else v->remotes[addrs[i]] = remote{};
        }
        v->reset(v->term);
        peers[id].r = v;
      } else {
        peers[id].r = nullptr;
      }
    }
  }
  raft* peer(u64 id) { return peers.at(id).r; }
  void send(std::vector<Message> msgs) {
    size_t head = 0;
    while (head < msgs.size()) {
      Message m = msgs[head++];
      raft* p = peers.at(m.To).r;
      if (!p) continue;
      p->Handle(m);
      auto out = filter(p->readMessages());
      for (auto& x : out) msgs.push_back(x);
    }
  }
  void send(const Message& m) { send(std::vector<Message>{m}); }
  void drop(u64 from, u64 to, double perc) { dropm[{from, to}] = perc; }
  void cut(u64 one, u64 other) { drop(one, other, 1); drop(other, one, 1); }
  void isolate(u64 id) {
    for (size_t i = 0; i < peers.size(); i++) {
      u64 nid = i + 1;
      if (nid != id) { drop(id, nid, 1.0); drop(nid, id, 1.0); }
    }
  }
  void ignore(MessageType t) { ignorem.insert(t); }
  void recover() { dropm.clear(); ignorem.clear(); }
  std::vector<Message> filter(std::vector<Message> msgs) {
    std::vector<Message> mm;
    for (auto& m : msgs) {
      if (ignorem.count(m.Type)) continue;
      if (m.Type == Election) panicf("unexpected msgHup");
      auto it = dropm.find({m.From, m.To});
      double perc = it == dropm.end() ? 0.0 : it->second;
      double n = (double)(rnd() >> 11) * (1.0 / 9007199254740992.0);
      if (n < perc) continue;
      mm.push_back(m);
    }
    return mm;
  }
};

inline Message Msg(u64 from, u64 to, MessageType t) {
  Message m;
  m.From = from;
  m.To = to;
  m.Type = t;
  return m;
}

inline Message PropMsg(u64 from, u64 to, const char* data) {
  Message m = Msg(from, to, Propose);
  Entry e;
  e.Cmd.assign(data, data + strlen(data));
  m.Entries.push_back(e);
  return m;
}

// --- minimal self-contained test runner -----------------------------------
struct TestCase {
  const char* name;
  void (*fn)();
};
inline std::vector<TestCase>& registry() {
  static std::vector<TestCase> r;
  return r;
}
struct Registrar {
  Registrar(const char* n, void (*f)()) { registry().push_back({n, f}); }
};
inline int& failures() {
  static int f = 0;
  return f;
}
#define KAT(name)                                  \
  static void name();                              \
  static ::oracle::Registrar reg_##name(#name, name); \
  static void name()
#define EXPECT(cond)                                                             \
  do {                                                                           \
    if (!(cond)) {                                                               \
      ::oracle::failures()++;                                                    \
      std::fprintf(stderr, "  %s:%d: expectation failed: %s\n", __FILE__, __LINE__, #cond); \
    }                                                                            \
  } while (0)
#define EXPECT_EQ(a, b)                                                                   \
  do {                                                                                    \
    auto _a = (a);                                                                        \
    auto _b = (b);                                                                        \
    if (!(_a == _b)) {                                                                    \
      ::oracle::failures()++;                                                             \
      std::fprintf(stderr, "  %s:%d: %s == %s failed (%llu vs %llu)\n", __FILE__, __LINE__, #a, #b, \
                   (unsigned long long)_a, (unsigned long long)_b);                       \
    }                                                                                     \
  } while (0)
#define EXPECT_PANIC(stmt)                                                                   \
  do {                                                                                       \
    bool _p = false;                                                                         \
    try { stmt; } catch (const ::oracle::Panic&) { _p = true; }                              \
    if (!_p) { ::oracle::failures()++;                                                       \
      std::fprintf(stderr, "  %s:%d: expected panic: %s\n", __FILE__, __LINE__, #stmt); }    \
  } while (0)

}  // namespace oracle
