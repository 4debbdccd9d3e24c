// batch.cpp — TEST INFRASTRUCTURE: the oracle as a population of faithful
// raft objects (raft_oracle.hpp) driven through the gpuraft record formats
// (include/gpuraft.h), so parity tests can feed identical inputs to the GPU
// engine and to the CPU restatement and compare every output.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
// this library (oracle/_build/liboracle.so). It is never part of the product.
//
// Per pass and per peer, inputs are applied in the engine's documented order,
// which is one of the orders node.stepNode can produce (node.go:652-780):
// messages grouped by sender slot (arrival order within a slot) through
// Peer.Handle (peer.go:199-209), then Peer.ReadIndex, Peer.Tick x n,
// Peer.QuiescedTick x n, Peer.ProposeEntries.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include "gpuraft.h"
#include "raft_oracle.hpp"

using namespace oracle;

namespace {

// A sparse ILogDB over term runs: the persisted log is [marker+1, last] with
// terms given by runs; entries are materialised on demand with a fixed
// payload size, so SizeUpperLimit() equals the host's entry_size_ub.
// Semantics follow TestLogDB (logdb_test.go:99-150).
struct RunLogDB : ILogDB {
  u64 marker = 0, markerTerm = 0, last = 0;
  std::vector<std::pair<u64, u64>> runs;  // (start, term), starts ascending, covering (marker, last]
  size_t payload = 16;
  State st;
  Snapshot snap;

  u64 termAt(u64 i) const {  // i in (marker, last]
    u64 t = runs.empty() ? markerTerm : runs[0].second;
    for (auto& r : runs)
      if (r.first <= i) t = r.second;
    return t;
  }
  std::pair<u64, u64> GetRange() override { return {marker + 1, last}; }
  State NodeState(Membership* m) override {
    if (m) *m = snap.membership;
    return st;
  }
  void SetState(const State& s) override { st = s; }
  Err CreateSnapshot(const Snapshot&) override { return Err::None; }
  Err ApplySnapshot(const Snapshot&) override { return Err::None; }
  Snapshot GetSnapshot() override { return snap; }
  u64 Term(u64 index, Err* err) override {
    *err = Err::None;
    if (index == marker) return markerTerm;
    auto e = Entries(index, index + 1, UINT64_MAX, err);
    if (*err != Err::None) return 0;
    if (e.empty()) return 0;
    return e[0].Term;
  }
  std::vector<Entry> Entries(u64 low, u64 high, u64 maxSize, Err* err) override {
    *err = Err::None;
    if (low <= marker) { *err = Err::Compacted; return {}; }
    if (high > last + 1) { *err = Err::Unavailable; return {}; }
    if (last == marker) { *err = Err::Unavailable; return {}; }
    std::vector<Entry> out;
    u64 total = 0;
    for (u64 i = low; i < high; i++) {
      Entry e;
      e.Index = i;
      e.Term = termAt(i);
      e.Cmd.assign(payload, 0);
      total += (u64)e.SizeUpperLimit();
      if (!out.empty() && total > maxSize) break;  // limitSize
      out.push_back(std::move(e));
    }
    return out;
  }
  Err Compact(u64) override { return Err::None; }
  Err Append(std::vector<Entry> es) override {
    if (es.empty()) return Err::None;
    u64 first = es[0].Index;
    if (first <= marker) panicf("RunLogDB append below marker");
    if (first > last + 1) panicf("RunLogDB hole");
    while (!runs.empty() && runs.back().first >= first) runs.pop_back();
    for (auto& e : es) {
      u64 prevTerm = runs.empty() ? (e.Index - 1 == marker ? markerTerm : ~0ull) : runs.back().second;
      if (runs.empty() || prevTerm != e.Term) runs.push_back({e.Index, e.Term});
    }
    last = es.back().Index;
    return Err::None;
  }
};

using u8 = uint8_t;

// Cache-line aligned: peers are stepped clusterID % T by T threads (the
// FixedPartitioner rule), so neighbouring records belong to different threads.
struct alignas(128) OPeer {
  std::unique_ptr<RunLogDB> db;
  std::unique_ptr<raft> r;
  std::vector<u64> ids;   // slot -> node id
  std::vector<u8> kinds;  // slot -> gr_slot_kind
  u64 entryUB = 0;
  std::vector<u64> rand;  // draws for the current pass
  size_t randNext = 0;
  u64 appendFrom = 0;
  uint32_t slotOf(u64 id) const {
    for (size_t j = 0; j < ids.size(); ++j)
      if (kinds[j] != GR_SLOT_EMPTY && ids[j] == id) return (uint32_t)j;
    return GR_SLOT_NONE;
  }
};

}  // namespace

// Long-lived workers, like dragonboat's step workers (execengine.go:122-129):
// worker t always steps the same peers (clusterID % T), so its allocations stay
// in its own malloc arena instead of bouncing between freshly created threads.
struct WorkerPool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable go, done;
  std::function<void(uint32_t)> job;
  uint64_t gen = 0;
  uint32_t pending = 0;
  bool quit = false;
  ~WorkerPool() { stop(); }
  void stop() {
    {
      std::lock_guard<std::mutex> g(mu);
      quit = true;
    }
    go.notify_all();
    for (auto& t : th) t.join();
    th.clear();
    quit = false;
  }
  void run(uint32_t n, const std::function<void(uint32_t)>& f) {
    if (th.size() != n) {
      stop();
      // a new worker starts having seen the current generation, so it waits for
      // this run's job and never picks up a previous (finished) one
      uint64_t g0;
      {
        std::lock_guard<std::mutex> g(mu);
        g0 = gen;
      }
      for (uint32_t t = 0; t < n; ++t) th.emplace_back([this, t, g0]() { loop(t, g0); });
    }
    std::unique_lock<std::mutex> g(mu);
    job = f;
    pending = n;
    gen++;
    go.notify_all();
    done.wait(g, [this]() { return pending == 0; });
    job = nullptr;  // f's captures belong to the caller's frame
  }
  void loop(uint32_t t, uint64_t seen) {
    for (;;) {
      std::function<void(uint32_t)> f;
      {
        std::unique_lock<std::mutex> g(mu);
        go.wait(g, [&]() { return quit || gen != seen; });
        if (quit) return;
        seen = gen;
        f = job;
      }
      f(t);
      std::lock_guard<std::mutex> g(mu);
      if (--pending == 0) done.notify_all();
    }
  }
};

struct ob_pop {
  uint32_t S = 0;
  WorkerPool pool;
  u64 maxEntrySize = MaxEntrySize;
  std::vector<OPeer> peers;
  std::vector<gr_message> lastOut;  // the last ob_step2 with out == NULL keeps its messages here
  std::vector<uint32_t> lastItems;
  // CPU-baseline mode only (ob_set_truncate_runs): a Replicate whose entries span
  // more than 2 term runs travels with the first two runs (a prefix of its
  // entries, as a size-limited send would). Parity runs keep it an error.
  bool truncateRuns = false;
};

namespace {

void build_peer(const gr_peer& g, uint32_t S, u64 maxEntrySize, OPeer* op) {
  op->db.reset(new RunLogDB());
  RunLogDB& db = *op->db;
  const u64 lo = g.first_index_m1, hi = g.last_index;
  db.marker = lo;
  db.last = hi;
  db.payload = g.entry_size_ub >= 128 ? (size_t)(g.entry_size_ub - 128) : 0;
  // term at lo: the first run if it starts at lo, else that run's term (the
  // region below the device window is filled with the oldest known term).
  db.markerTerm = g.n_runs ? g.run_term[0] : 0;
  for (int k = 0; k < g.n_runs; ++k) {
    u64 s = std::max(g.run_start[k], lo + 1);
    if (s > hi) continue;
    if (!db.runs.empty() && db.runs.back().first == s) db.runs.back().second = g.run_term[k];
    else db.runs.push_back({s, g.run_term[k]});
  }
  Config c;
  c.NodeID = g.node_id;
  c.ElectionRTT = g.election_timeout;
  c.HeartbeatRTT = g.heartbeat_timeout;
  c.CheckQuorum = (g.flags & GR_F_CHECK_QUORUM) != 0;
  c.IsObserver = g.state == GR_OBSERVER;
  OPeer* self = op;
  op->r.reset(new raft(c, &db, [self]() -> u64 {
    u64 v;
    if (self->randNext < self->rand.size()) v = self->rand[self->randNext];
    else v = SplitMix64(self->rand.empty() ? 7 : self->rand.back() + self->randNext)();
    self->randNext++;
    return v;
  }));
  raft& r = *op->r;
  r.maxEntrySize = maxEntrySize;
  r.term = g.term;
  r.vote = g.vote;
  r.log->committed = g.committed;
  r.log->applied = lo;
  r.applied = g.applied;
  r.state = (RaftState)g.state;
  r.leaderID = g.leader_id;
  r.leaderTransferTarget = g.leader_transfer_target;
  r.isLeaderTransferTarget = (g.flags & GR_F_IS_LEADER_TRANSFER_TARGET) != 0;
  r.pendingConfigChange = (g.flags & GR_F_PENDING_CONFIG_CHANGE) != 0;
  r.checkQuorum = (g.flags & GR_F_CHECK_QUORUM) != 0;
  r.electionTick = g.election_tick;
  r.heartbeatTick = g.heartbeat_tick;
  r.randomizedElectionTimeout = g.randomized_election_timeout;
  r.electionTimeout = g.election_timeout;
  r.heartbeatTimeout = g.heartbeat_timeout;
  r.remotes.clear();
  r.observers.clear();
  op->ids.assign(S, 0);
  op->kinds.assign(S, GR_SLOT_EMPTY);
  for (uint32_t j = 0; j < S; ++j) {
    op->ids[j] = g.remote_id[j];
    op->kinds[j] = g.remotes[j].kind;
    if (g.remotes[j].kind == GR_SLOT_EMPTY) continue;
    remote rm;
    rm.match = g.remotes[j].match;
    rm.next = g.remotes[j].next;
    rm.snapshotIndex = g.remotes[j].snapshot_index;
    rm.state = (remoteStateType)g.remotes[j].state;
    rm.active = g.remotes[j].active != 0;
    if (g.remotes[j].kind == GR_SLOT_VOTER) r.remotes[g.remote_id[j]] = rm;
    else r.observers[g.remote_id[j]] = rm;
  }
  r.resetMatchValueArray();
  r.readIdx = readIndex{};
  for (int q = 0; q < g.read_index_count; ++q) {
    const gr_read_status& rs = g.read_index[q];
    SystemCtx ctx{rs.ctx_low, rs.ctx_high};
    auto s = std::make_shared<readStatus>();
    s->index = rs.index;
    s->from = rs.from_slot == GR_SLOT_NONE ? 0 : g.remote_id[rs.from_slot];
    s->ctx = ctx;
    for (uint32_t j = 0; j < S; ++j)
      if (rs.ack_bits & (1u << j)) s->confirmed[g.remote_id[j]] = true;
    r.readIdx.queue.push_back(ctx);
    r.readIdx.pending[ctx] = s;
  }
  r.msgs.clear();
  r.readyToRead.clear();
  op->entryUB = g.entry_size_ub;
  r.log->onTryAppend = [op](u64 ci) { op->appendFrom = op->appendFrom ? std::min(op->appendFrom, ci) : ci; };
  // The in-memory log's persistence marks (gpuraft.h gr_peer.saved_to / marker_index /
  // log_applied); marker_index == 0 keeps newEntryLog's (inmem at lastIndex + 1).
  if (g.marker_index != 0) {
    inMemory& im = r.log->inmem;
    im.markerIndex = g.marker_index;
    im.savedTo = g.saved_to;
    im.entries.clear();
    for (u64 i = g.marker_index; i <= hi; ++i) {
      Entry e;
      e.Index = i;
      e.Term = db.termAt(i);
      e.Cmd.assign(db.payload, 0);
      im.entries.push_back(std::move(e));
    }
    r.log->applied = g.log_applied;
  }
}

// Term runs of the oracle log over [lo, hi] (lo = firstIndex-1): the logdb
// part below the in-memory marker, then the in-memory entries.
std::vector<std::pair<u64, u64>> log_runs(const OPeer& op) {
  const entryLog& l = *op.r->log;
  const u64 lo = l.firstIndex() - 1, hi = l.lastIndex();
  std::vector<std::pair<u64, u64>> runs;
  auto add = [&](u64 idx, u64 t) {
    if (runs.empty() || runs.back().second != t) runs.push_back({idx, t});
  };
  Err e;
  add(lo, l.term(lo, &e));
  const u64 mark = l.inmem.markerIndex;
  const RunLogDB& db = *op.db;
  const u64 dbTop = std::min(hi, mark - 1);
  for (auto& rr : db.runs) {
    if (rr.first > dbTop) break;
    u64 nextStart = dbTop + 1;
    for (auto& r2 : db.runs)
      if (r2.first > rr.first) { nextStart = r2.first; break; }
    if (nextStart <= lo + 1) continue;
    add(std::max(rr.first, lo + 1), rr.second);
  }
  for (auto& en : l.inmem.entries)
    if (en.Index > lo && en.Index <= hi) add(en.Index, en.Term);
  return runs;
}

void export_peer(const OPeer& op, uint32_t S, gr_peer* g) {
  const raft& r = *op.r;
  memset(g, 0, sizeof(*g));
  g->term = r.term;
  g->vote = r.vote;
  g->committed = r.log->committed;
  g->applied = r.applied;
  g->last_index = r.log->lastIndex();
  g->first_index_m1 = r.log->firstIndex() - 1;
  g->leader_id = r.leaderID;
  g->leader_transfer_target = r.leaderTransferTarget;
  g->node_id = r.nodeID;
  g->election_tick = r.electionTick;
  g->heartbeat_tick = r.heartbeatTick;
  g->randomized_election_timeout = r.randomizedElectionTimeout;
  g->election_timeout = r.electionTimeout;
  g->heartbeat_timeout = r.heartbeatTimeout;
  g->entry_size_ub = op.entryUB;
  g->saved_to = r.log->inmem.savedTo;
  g->marker_index = r.log->inmem.markerIndex;
  g->log_applied = r.log->applied;
  auto runs = log_runs(op);
  size_t first = runs.size() > GR_K ? runs.size() - GR_K : 0;
  g->n_runs = (uint8_t)(runs.size() - first);
  for (size_t k = first; k < runs.size(); ++k) {
    g->run_start[k - first] = runs[k].first;
    g->run_term[k - first] = runs[k].second;
  }
  g->state = (uint8_t)r.state;
  g->flags = (uint8_t)((r.checkQuorum ? GR_F_CHECK_QUORUM : 0) |
                       (r.isLeaderTransferTarget ? GR_F_IS_LEADER_TRANSFER_TARGET : 0) |
                       (r.pendingConfigChange ? GR_F_PENDING_CONFIG_CHANGE : 0));
  g->self_slot = GR_SLOT_NONE;
  for (uint32_t j = 0; j < S; ++j) {
    g->remote_id[j] = op.ids[j];
    const remote* rm = nullptr;
    auto it = r.remotes.find(op.ids[j]);
    auto ot = r.observers.find(op.ids[j]);
    uint8_t kind = GR_SLOT_EMPTY;
    if (op.kinds[j] != GR_SLOT_EMPTY && it != r.remotes.end()) { rm = &it->second; kind = GR_SLOT_VOTER; }
    else if (op.kinds[j] != GR_SLOT_EMPTY && ot != r.observers.end()) { rm = &ot->second; kind = GR_SLOT_OBSERVER; }
    g->remotes[j].kind = kind;
    if (rm) {
      g->remotes[j].match = rm->match;
      g->remotes[j].next = rm->next;
      g->remotes[j].snapshot_index = rm->snapshotIndex;
      g->remotes[j].state = (uint8_t)rm->state;
      g->remotes[j].active = rm->active ? 1 : 0;
      if (op.ids[j] == r.nodeID) g->self_slot = (uint8_t)j;
    }
  }
  int q = 0;
  for (auto& ctx : r.readIdx.queue) {
    if (q >= GR_Q) break;
    auto s = r.readIdx.pending.at(ctx);
    gr_read_status& rs = g->read_index[q++];
    rs.index = s->index;
    rs.ctx_low = ctx.Low;
    rs.ctx_high = ctx.High;
    rs.from_slot = s->from == 0 ? GR_SLOT_NONE : (uint8_t)op.slotOf(s->from);
    uint8_t ack = 0;
    for (auto& kv : s->confirmed) {
      uint32_t j = op.slotOf(kv.first);
      if (j != GR_SLOT_NONE) ack |= (uint8_t)(1u << j);
    }
    rs.ack_bits = ack;
  }
  g->read_index_count = (uint8_t)q;
}

// raftpb.Message -> gr_message (target slot, entries as term runs).
bool to_record(const OPeer& op, uint32_t peer, const Message& m, gr_message* o, bool truncate_runs = false) {
  memset(o, 0, sizeof(*o));
  o->peer = peer;
  o->type = (uint8_t)m.Type;
  o->slot = (uint8_t)op.slotOf(m.To);
  o->reject = m.Reject ? 1 : 0;
  o->term = m.Term;
  o->log_index = m.LogIndex;
  o->log_term = m.LogTerm;
  o->commit = m.Commit;
  o->hint = m.Hint;
  o->hint_high = m.HintHigh;
  o->n_entries = (uint32_t)m.Entries.size();
  if (m.Type == Propose)  // a Propose record's reject bit: the batch holds a ConfigChangeEntry
    for (const Entry& e : m.Entries) o->reject |= e.Type == ConfigChangeEntry ? 1 : 0;
  bool ok = o->slot != GR_SLOT_NONE;
  if (!m.Entries.empty()) {
    o->n_runs = 1;
    o->run_term[0] = m.Entries[0].Term;
    for (size_t k = 1; k < m.Entries.size(); ++k) {
      if (m.Entries[k].Term != m.Entries[k - 1].Term) {
        if (o->n_runs == 2) {
          if (truncate_runs) o->n_entries = (uint32_t)k;
          else ok = false;
          break;
        }
        o->n_runs = 2;
        o->run2_offset = (uint32_t)k;
        o->run_term[1] = m.Entries[k].Term;
      }
    }
  }
  return ok;
}

Message from_record(const OPeer& op, const gr_message& g) {
  Message m;
  m.Type = (MessageType)g.type;
  m.From = op.ids[g.slot];
  m.To = op.r->nodeID;
  m.Term = g.term;
  m.LogIndex = g.log_index;
  m.LogTerm = g.log_term;
  m.Commit = g.commit;
  m.Reject = g.reject != 0;
  m.Hint = g.hint;
  m.HintHigh = g.hint_high;
  const size_t payload = op.entryUB >= 128 ? (size_t)(op.entryUB - 128) : 0;
  for (uint32_t k = 0; k < g.n_entries; ++k) {
    Entry e;
    e.Index = g.log_index + 1 + k;
    e.Term = (g.n_runs == 2 && k >= g.run2_offset) ? g.run_term[1] : g.run_term[0];
    e.Cmd.assign(payload, 0);
    m.Entries.push_back(std::move(e));
  }
  if (m.Type == Propose && m.Reject) {  // see to_record
    m.Reject = false;
    if (!m.Entries.empty()) m.Entries[0].Type = ConfigChangeEntry;
  }
  return m;
}

// ---- escalation predicate -------------------------------------------------
// The device escalates an item (hands it to the host) for a reason (gr_escalation).
// The harness re-derives, from the oracle's own execution of that item, every
// reason that applies to it, so a test can fail any escalation the reference
// behaviour does not justify (too early, or for the wrong reason). The device's
// term-run window is modelled here (same truncate/push rules as gr_lane.h) from
// the device state at the start of the pass.
struct ItemProbe : Probe {
  std::vector<std::pair<u64, u64>> runs;  // device window model: (start, term), <= GR_K
  bool active = false;
  bool termWindow = false, replErr = false, riCap = false;
  int resetsPass = 0, resetsItem = 0, campaigns = 0;
  u64 replMaxCnt = 0;
  void begin_item() {
    termWindow = replErr = riCap = false;
    resetsItem = campaigns = 0;
    replMaxCnt = 0;
  }
  void lookup(u64 i) override {
    if (active && (runs.empty() || i < runs[0].first)) termWindow = true;
  }
  void merged(const std::vector<Entry>& es) override {
    if (es.empty()) return;
    const u64 ci = es[0].Index;
    while (!runs.empty() && runs.back().first >= ci) runs.pop_back();  // win_truncate
    for (const Entry& e : es) {                                          // win_push per term change
      if (!runs.empty() && runs.back().second == e.Term) continue;
      if (runs.size() == GR_K) runs.erase(runs.begin());
      runs.push_back({e.Index, e.Term});
    }
  }
  void resetCalled() override {
    resetsPass++;
    if (active) resetsItem++;
  }
  void campaignCalled() override {
    if (active) campaigns++;
  }
  void replicateError() override {
    if (active) replErr = true;
  }
  void replicateRange(u64 next, u64 last) override {
    if (active && next <= last) replMaxCnt = std::max<u64>(replMaxCnt, last - next + 1);
  }
  void readIndexAdd(size_t queued, bool dup) override {
    if (active && !dup && queued >= GR_Q) riCap = true;
  }
};

inline bool wide64(u64 a) { return (a >> 32) != 0; }

// UNSUPPORTED: (state, message) pairs the device hands to the host
// (gr_lane.h Lane::handle and its handlers), from the oracle's state at the item.
bool unsupported_msg(const raft& r, const Message& m, bool fwd_before) {
  const MessageType t = m.Type;
  RaftState st = r.state;
  if (m.Term != 0 && m.Term != r.term) {
    if (m.Term < r.term) return false;  // dropped or answered with NoOP
    if (t == RequestVote) return true;
    if (st != observer) {
      if (fwd_before) return true;      // step-down after forwarded proposals were appended
      st = follower;
    }
  }
  if (st == leader) {
    if (t == RequestVote) return true;
    if (t == Propose) {
      bool transferring = r.leaderTransferTarget != NoNode;
      return m.Entries.empty() || r.selfRemoved() || transferring;
    }
    return false;
  }
  if (st == follower || st == observer) {
    if (t == InstallSnapshot) return true;
    if ((t == RequestVote || t == TimeoutNow) && st != observer) return true;
    return false;
  }
  return t == Heartbeat || t == Replicate || t == InstallSnapshot || t == RequestVoteResp || t == Election ||
         t == RequestVote;  // candidate
}

}  // namespace

extern "C" {

int ob_create(uint32_t slots, uint64_t max_entry_size, const gr_peer* peers, uint32_t n, ob_pop** out) {
  if (!out || (n && !peers) || slots == 0 || slots > GR_SMAX) return GR_EINVAL;
  ob_pop* p = new ob_pop();
  p->S = slots;
  p->maxEntrySize = max_entry_size;
  p->peers.resize(n);
  try {
    for (uint32_t k = 0; k < n; ++k) build_peer(peers[k], slots, max_entry_size, &p->peers[k]);
  } catch (const std::exception&) {
    delete p;
    return GR_ESTATE;
  }
  *out = p;
  return GR_OK;
}

void ob_destroy(ob_pop* p) { delete p; }

// Rebuild one peer from a record (state injections in simulations).
int ob_reload(ob_pop* p, uint32_t peer, const gr_peer* rec) {
  if (!p || !rec || peer >= p->peers.size()) return GR_EINVAL;
  try {
    build_peer(*rec, p->S, p->maxEntrySize, &p->peers[peer]);
  } catch (const std::exception&) {
    return GR_ESTATE;
  }
  return GR_OK;
}

// 1 if the peer's state fits a gr_peer record exactly (the device can hold
// it), 0 if the host must keep stepping it: more than GR_Q pending ReadIndex
// requests, or members outside the slot table.
int ob_representable(ob_pop* p, uint8_t* out, uint32_t n) {
  if (!p || n > p->peers.size()) return GR_EINVAL;
  for (uint32_t k = 0; k < n; ++k) {
    const OPeer& op = p->peers[k];
    const raft& r = *op.r;
    bool ok = r.readIdx.queue.size() <= GR_Q && r.readIdx.pending.size() <= GR_Q;
    for (auto& kv : r.remotes) ok = ok && op.slotOf(kv.first) != GR_SLOT_NONE;
    for (auto& kv : r.observers) ok = ok && op.slotOf(kv.first) != GR_SLOT_NONE;
    out[k] = ok ? 1 : 0;
  }
  return GR_OK;
}

// entryLog.commitUpdate (logentry.go:325-335) for a slot list, as gr_commit_update:
// status 1 where the reference panics ("invalid applyto"), and such a slot is left
// untouched.
int ob_commit_update(ob_pop* p, const uint32_t* slots, const gr_update_commit* uc, uint32_t n, int32_t* status) {
  if (!p) return GR_EINVAL;
  int rc = GR_OK;
  for (uint32_t x = 0; x < n; ++x) {
    if (slots[x] >= p->peers.size()) return GR_ERANGE;
    entryLog& l = *p->peers[slots[x]].r->log;
    const gr_update_commit& u = uc[x];
    if (u.applied_to > 0 && (u.applied_to < l.applied || u.applied_to > l.committed)) {
      status[x] = 1;
      rc = GR_ESTATE;
      continue;
    }
    UpdateCommit c;
    c.StableLogTo = u.stable_log_to;
    c.StableLogTerm = u.stable_log_term;
    c.AppliedTo = u.applied_to;
    l.commitUpdate(c);
    status[x] = 0;
  }
  return rc;
}

int ob_set_truncate_runs(ob_pop* p, int on) {
  if (!p) return GR_EINVAL;
  p->truncateRuns = on != 0;
  return GR_OK;
}

int ob_export(ob_pop* p, gr_peer* out, uint32_t n) {
  if (!p || n > p->peers.size()) return GR_EINVAL;
  for (uint32_t k = 0; k < n; ++k) export_peer(p->peers[k], p->S, &out[k]);
  return GR_OK;
}

// Persist and apply everything after a pass (node.go processRaftUpdate /
// Peer.Commit): entriesToSave -> LogDB, StableLogTo, AppliedTo = committed,
// NotifyRaftLastApplied(committed). Keeps in-memory logs bounded in long runs.
static void commit_peer(OPeer& op) {
  {
    raft& r = *op.r;
    auto es = r.log->entriesToSave();
    if (!es.empty()) {
      op.db->Append(es);
      UpdateCommit uc;
      uc.StableLogTo = es.back().Index;
      uc.StableLogTerm = es.back().Term;
      r.log->commitUpdate(uc);
    }
    if (r.log->committed > r.log->applied) {
      UpdateCommit ac;
      ac.AppliedTo = r.log->committed;
      r.log->commitUpdate(ac);
    }
    r.applied = r.log->committed;
  }
}

int ob_commit_all(ob_pop* p) {
  if (!p) return GR_EINVAL;
  for (auto& op : p->peers) commit_peer(op);
  return GR_OK;
}

// ob_commit_all on the step's partition (peer p on worker p % T, as ob_step2
// with n_threads = T): each worker frees and reallocates the log memory of its
// own peers, so its allocations stay in its own malloc arena instead of
// bouncing through the arena of the thread that first built them.
int ob_commit_all_mt(ob_pop* p, uint32_t n_threads) {
  if (!p) return GR_EINVAL;
  if (n_threads <= 1) return ob_commit_all(p);
  const uint32_t n = (uint32_t)p->peers.size();
  p->pool.run(n_threads, [&](uint32_t t) {
    for (uint32_t pi = t; pi < n; pi += n_threads) commit_peer(p->peers[pi]);
  });
  return GR_OK;
}

// Rebuild every peer from its own record on the worker that will step it
// (partition p % T): the CPU baseline's per-thread heaps start out local too.
int ob_rehome(ob_pop* p, uint32_t n_threads) {
  if (!p) return GR_EINVAL;
  if (n_threads <= 1) return GR_OK;
  const uint32_t n = (uint32_t)p->peers.size();
  std::vector<gr_peer> recs(n);
  for (uint32_t k = 0; k < n; ++k) export_peer(p->peers[k], p->S, &recs[k]);
  std::atomic<int> bad{0};
  p->pool.run(n_threads, [&](uint32_t t) {
    for (uint32_t pi = t; pi < n; pi += n_threads) {
      try {
        build_peer(recs[pi], p->S, p->maxEntrySize, &p->peers[pi]);  // frees the old objects here
      } catch (const std::exception&) {
        bad = 1;
      }
    }
  });
  return bad ? GR_ESTATE : GR_OK;
}

// One pass over the population. For peer p, items are numbered as the engine
// numbers them (messages, ReadIndex, ticks, one quiesced-tick item, propose).
// If limits != NULL, mid[p] receives the state after items < limits[p] and
// results/ready reflect only that prefix; messages carry the emitting item
// index in out_item so callers can split device-prefix and host-suffix output.
// esc_mask (may be NULL) receives, for every peer with a limit, the set of
// gr_escalation reasons (bit r) the item at limits[p] justifies; dev_before
// (may be NULL: the oracle's own export is used) is the device state at the
// start of the pass, whose term-run window the predicate models; in_depth /
// out_depth are the mailbox depths of the device spaces; has_locals = 0 models
// a device pass without local-input rows (every reset() needs the host).
// n_threads > 1 steps disjoint peer ranges concurrently (clusterID % T, the
// FixedPartitioner rule of internal/server/partition.go:34-36).
int ob_step2(ob_pop* p, const gr_inbox* in, const uint32_t* limits, const gr_peer* dev_before, uint32_t in_depth,
             uint32_t out_depth, uint32_t has_locals, uint32_t* esc_mask, gr_peer* mid, gr_message* out,
             uint32_t* out_item, size_t cap, size_t* n_out, gr_peer_result* results, uint32_t n_threads, char* err,
             size_t errcap) {
  if (!p || !in || !n_out) return GR_EINVAL;
  const uint32_t n = (uint32_t)p->peers.size(), S = p->S;
  if (in_depth == 0) in_depth = GR_C;
  if (out_depth == 0) out_depth = GR_C;
  // bucket messages per (peer, slot), arrival order kept: a counting sort
  std::vector<uint32_t> start((size_t)n * S + 1, 0), order(in->n_msgs);
  for (size_t k = 0; k < in->n_msgs; ++k) {
    const gr_message& m = in->msgs[k];
    if (m.peer >= n || m.slot >= S) return GR_EINVAL;
    start[(size_t)m.peer * S + m.slot + 1]++;
  }
  for (size_t x = 1; x < start.size(); ++x) start[x] += start[x - 1];
  {
    std::vector<uint32_t> fill(start.begin(), start.end() - 1);
    for (size_t k = 0; k < in->n_msgs; ++k) {
      const gr_message& m = in->msgs[k];
      order[fill[(size_t)m.peer * S + m.slot]++] = (uint32_t)k;
    }
  }
  std::vector<const gr_local_input*> loc(n, nullptr);
  for (size_t k = 0; k < in->n_locals; ++k) {
    if (in->locals[k].peer >= n) return GR_EINVAL;
    loc[in->locals[k].peer] = &in->locals[k];
  }
  struct Out {
    uint32_t peer, item;
    gr_message rec;
    bool ok;
  };
  if (n_threads == 0) n_threads = 1;
  struct alignas(128) PerThread {  // one cache line apart: no false sharing between workers
    std::vector<Out> v;
  };
  std::vector<PerThread> outv(n_threads);
  std::vector<std::string> errs(n_threads);
  static const bool kTime = getenv("GR_OB_TIMING") != nullptr;  // TEMP
  std::vector<double> tw(n_threads, 0);
  auto t_all0 = std::chrono::steady_clock::now();
  auto work = [&](uint32_t t) {
    auto tw0 = std::chrono::steady_clock::now();
    struct TW { std::vector<double>& v; uint32_t t; std::chrono::steady_clock::time_point a;
      ~TW() { v[t] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count(); } } twg{tw, t, tw0};
    ItemProbe probe;
    g_probe = &probe;
    for (uint32_t pi = t; pi < n; pi += n_threads) {
      OPeer& op = p->peers[pi];
      raft& r = *op.r;
      const uint32_t limit = limits ? limits[pi] : 0xFFFFFFFFu;
      const bool want_mask = esc_mask && limit != 0xFFFFFFFFu;
      r.msgs.clear();
      r.readyToRead.clear();
      op.appendFrom = 0;
      op.rand.clear();
      op.randNext = 0;
      // the draw is an input: a peer without a local record gets the device's zero row
      if (has_locals) op.rand.push_back(loc[pi] ? loc[pi]->rand : 0);
      probe.runs.clear();
      probe.active = false;
      probe.resetsPass = 0;
      if (want_mask) {
        gr_peer w;
        if (dev_before) w = dev_before[pi];
        else export_peer(op, S, &w);
        for (int k = 0; k < w.n_runs && k < GR_K; ++k) probe.runs.push_back({w.run_start[k], w.run_term[k]});
      }
      uint32_t item = 0;
      uint32_t mask = 0;
      std::vector<uint32_t> sent(S, 0);  // messages this peer emitted per target slot
      gr_peer_result res;
      memset(&res, 0, sizeof(res));
      res.peer = pi;
      bool midTaken = false;
      auto take_mid = [&]() {
        if (midTaken) return;
        midTaken = true;
        if (mid) export_peer(op, S, &mid[pi]);
        res.n_ready = (uint8_t)std::min<size_t>(r.readyToRead.size(), 255);
        for (size_t q = 0; q < r.readyToRead.size() && q < GR_Q; ++q) {
          res.ready[q].index = r.readyToRead[q].Index;
          res.ready[q].ctx_low = r.readyToRead[q].ctx.Low;
          res.ready[q].ctx_high = r.readyToRead[q].ctx.High;
        }
        res.append_from = op.appendFrom;
        // getUpdate (peer.go:311-337): the log marks and raftState() after the prefix
        res.committed = r.log->committed;
        res.last_index = r.log->lastIndex();
        auto es = r.log->entriesToSave();
        res.save_from = es.empty() ? 0 : es.front().Index;
        res.term = r.term;
        res.vote = r.vote;
      };
      // called before item `it` runs: arms the probe for the escalated item
      auto pre = [&](uint32_t it) {
        if (it == limit) take_mid();
        probe.active = want_mask && it == limit;
        if (probe.active) probe.begin_item();
      };
      // after item `it`: its messages; for the escalated item, the reasons
      auto flush = [&](uint32_t it) {
        const bool judged = probe.active;
        for (auto& m : r.msgs) {
          Out o;
          o.peer = pi;
          o.item = it;
          o.ok = to_record(op, pi, m, &o.rec, p->truncateRuns);
          if (o.rec.slot < S) sent[o.rec.slot]++;
          if (judged) {
            if (op.slotOf(m.To) == GR_SLOT_NONE) mask |= 1u << GR_ESC_NONMEMBER;
            else if (sent[o.rec.slot] > out_depth) mask |= 1u << GR_ESC_CAPACITY;
            u64 rt1 = 0;
            int runs = m.Entries.empty() ? 0 : 1;
            for (size_t k = 1; k < m.Entries.size(); ++k)
              if (m.Entries[k].Term != m.Entries[k - 1].Term) { runs++; rt1 = std::max<u64>(rt1, m.Entries[k].Term); }
            if (runs > 2) mask |= 1u << GR_ESC_MSG_RUNS;
            const u64 mterm = isRequestMessage(m.Type) ? m.Term : r.term;
            if (wide64(mterm) || wide64(m.LogTerm) || (!m.Entries.empty() && wide64(m.Entries[0].Term)) || wide64(rt1))
              mask |= 1u << GR_ESC_WIDE_TERM;
          }
          outv[t].v.push_back(o);
        }
        r.msgs.clear();
        if (judged) {
          if (probe.termWindow) mask |= 1u << GR_ESC_TERM_WINDOW;
          if (probe.resetsItem && (probe.resetsPass > probe.resetsItem || !has_locals)) mask |= 1u << GR_ESC_RANDOM;
          if (probe.campaigns) mask |= 1u << GR_ESC_ELECTION;
          if (probe.replErr) mask |= 1u << GR_ESC_SNAPSHOT;
          if (probe.replMaxCnt > 1 &&
              (op.entryUB == 0 || probe.replMaxCnt > p->maxEntrySize / op.entryUB))
            mask |= 1u << GR_ESC_ENTRY_SIZE;
          if (probe.replMaxCnt > 0xFFFFFFFFull || probe.riCap || r.readyToRead.size() > GR_Q)
            mask |= 1u << GR_ESC_CAPACITY;
          probe.active = false;
        }
      };
      try {
        for (uint32_t j = 0; j < S; ++j) {
          const size_t b0 = start[(size_t)pi * S + j], b1 = start[(size_t)pi * S + j + 1];
          for (size_t x = b0; x < b1; ++x) {
            const gr_message* gm = &in->msgs[order[x]];
            pre(item);
            Message m = from_record(op, *gm);
            if (probe.active) {
              if (x - b0 >= in_depth) mask |= 1u << GR_ESC_CAPACITY;  // did not fit the mailbox
              if (wide64(m.Term) || wide64(m.LogTerm) || (gm->n_runs && wide64(gm->run_term[0])) ||
                  (gm->n_runs == 2 && wide64(gm->run_term[1])))
                mask |= 1u << GR_ESC_WIDE_TERM;
              bool member = op.kinds[j] != GR_SLOT_EMPTY;
              if ((member || !isResponseMessageType(m.Type)) && unsupported_msg(r, m, res.n_forwarded != 0))
                mask |= 1u << GR_ESC_UNSUPPORTED;
              if (m.Type == Propose && gm->reject && r.state == leader) mask |= 1u << GR_ESC_CONFIG_CHANGE;
            }
            const u64 before = r.log->lastIndex();
            const RaftState st0 = r.state;
            // Peer.Handle (peer.go:199-209)
            bool member = op.kinds[j] != GR_SLOT_EMPTY;
            if (member || !isResponseMessageType(m.Type)) r.Handle(m);
            if (probe.active && st0 == leader && r.state != leader && res.n_forwarded) mask |= 1u << GR_ESC_UNSUPPORTED;
            if (m.Type == Propose && !midTaken && r.log->lastIndex() > before) {  // forwarded batch appended
              if (!res.propose_first) res.propose_first = before + 1;
              res.n_forwarded++;
              res.forwarded_entries += (uint32_t)m.Entries.size();
            }
            flush(item);
            item++;
          }
        }
        const gr_local_input* L = loc[pi];
        if (L) {
          if (L->read_index) {
            pre(item);
            SystemCtx ctx{L->read_ctx_low, L->read_ctx_high};
            Message m;
            m.Type = ReadIndex;
            m.Hint = ctx.Low;
            m.HintHigh = ctx.High;
            r.Handle(m);  // Peer.ReadIndex (peer.go:262-269)
            flush(item);
            item++;
          }
          for (uint32_t k = 0; k < L->ticks; ++k) {
            pre(item);
            const RaftState st0 = r.state;
            r.tick();
            if (probe.active && st0 == leader && r.state != leader && res.n_forwarded) mask |= 1u << GR_ESC_UNSUPPORTED;
            flush(item);
            item++;
          }
          if (L->quiesced_ticks) {
            pre(item);
            for (uint32_t k = 0; k < L->quiesced_ticks; ++k) r.quiescedTick();
            flush(item);
            item++;
          }
          if (L->propose_entries) {
            pre(item);
            const u64 before = r.log->lastIndex();
            std::vector<Entry> es(L->propose_entries);
            const size_t payload = op.entryUB >= 128 ? (size_t)(op.entryUB - 128) : 0;
            for (auto& e : es) e.Cmd.assign(payload, 0);
            if (L->propose_has_config_change) es[0].Type = ConfigChangeEntry;
            if (probe.active && L->propose_has_config_change && r.state == leader && !r.selfRemoved() &&
                r.leaderTransferTarget == NoNode)
              mask |= 1u << GR_ESC_CONFIG_CHANGE;
            Message m;
            m.Type = Propose;
            m.From = r.nodeID;
            m.Entries = es;
            r.Handle(m);  // Peer.ProposeEntries (peer.go:126-134)
            bool fwd = false;
            for (auto& x : r.msgs) fwd = fwd || x.Type == Propose;
            flush(item);
            if (!midTaken) {
              if (r.log->lastIndex() > before) {
                res.propose_result = GR_PROP_APPENDED;
                if (!res.propose_first) res.propose_first = before + 1;
              } else {
                res.propose_result = fwd ? GR_PROP_FORWARDED : GR_PROP_DROPPED;
              }
            }
            item++;
          }
        }
        take_mid();
      } catch (const std::exception& ex) {
        if (errs[t].empty()) errs[t] = "peer " + std::to_string(pi) + " item " + std::to_string(item) + ": " + ex.what();
        if (probe.active) {
          mask |= 1u << GR_ESC_PANIC;
          if (probe.replErr) mask |= 1u << GR_ESC_SNAPSHOT;  // the snapshot path itself panicked
          if (probe.termWindow) mask |= 1u << GR_ESC_TERM_WINDOW;
          if (probe.campaigns) mask |= 1u << GR_ESC_ELECTION;
          probe.active = false;
        }
        r.msgs.clear();
        take_mid();
        res.escalation = GR_ESC_PANIC;
        res.esc_item = item;
      }
      if (results) results[pi] = res;
      if (esc_mask) esc_mask[pi] = want_mask ? mask : 0;
    }
    g_probe = nullptr;
  };
  auto t_w0 = std::chrono::steady_clock::now();
  if (n_threads == 1) work(0);
  else p->pool.run(n_threads, work);
  if (kTime) {
    auto t_w1 = std::chrono::steady_clock::now();
    fprintf(stderr, "ob_step2: pre %.2f ms, run %.2f ms, threads:", std::chrono::duration<double, std::milli>(t_w0 - t_all0).count(),
            std::chrono::duration<double, std::milli>(t_w1 - t_w0).count());
    for (double x : tw) fprintf(stderr, " %.1f", x);
    fprintf(stderr, "\n");
  }
  size_t k = 0;
  bool bad = false;
  if (!out) {  // kept for ob_fetch_out (the caller sizes its buffers exactly)
    size_t tot = 0;
    for (auto& pt : outv) tot += pt.v.size();
    p->lastOut.resize(tot);
    p->lastItems.resize(tot);
  }
  for (auto& pt : outv) {
    for (auto& o : pt.v) {
      if (out && k < cap) {
        out[k] = o.rec;
        if (out_item) out_item[k] = o.item;
      } else if (!out) {
        p->lastOut[k] = o.rec;
        p->lastItems[k] = o.item;
      }
      if (!o.ok) bad = true;
      k++;
    }
  }
  *n_out = k;
  std::string e;
  for (auto& s : errs)
    if (!s.empty()) { e = s; break; }
  if (bad && e.empty()) e = "message not representable as a gr_message record";
  if (err && errcap) {
    strncpy(err, e.c_str(), errcap - 1);
    err[errcap - 1] = 0;
  }
  if (k > cap && out) return GR_ECAPACITY;
  return e.empty() ? GR_OK : GR_ESTATE;
}

// The messages of the last ob_step2 called with out == NULL.
int ob_fetch_out(ob_pop* p, gr_message* out, uint32_t* items, size_t cap) {
  if (!p || (cap && (!out || !items)) || cap < p->lastOut.size()) return GR_EINVAL;
  if (!p->lastOut.empty()) {
    memcpy(out, p->lastOut.data(), p->lastOut.size() * sizeof(gr_message));
    memcpy(items, p->lastItems.data(), p->lastItems.size() * sizeof(uint32_t));
  }
  p->lastOut.clear();
  p->lastItems.clear();
  return GR_OK;
}

int ob_step(ob_pop* p, const gr_inbox* in, const uint32_t* limits, gr_peer* mid, gr_message* out,
            uint32_t* out_item, size_t cap, size_t* n_out, gr_peer_result* results, uint32_t n_threads,
            char* err, size_t errcap) {
  return ob_step2(p, in, limits, nullptr, GR_C, GR_C, 1, nullptr, mid, out, out_item, cap, n_out, results, n_threads,
                  err, errcap);
}

}  // extern "C"
