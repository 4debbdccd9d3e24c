// raft_oracle.hpp — CPU restatement of dragonboat's internal/raft step.
//
// TEST INFRASTRUCTURE ONLY. This file is the parity oracle for the gpuraft
// engine. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
// may build, load or call it; the product library (libgpuraft.so) never links
// it and has no CPU fallback.
//
// It restates, function by function, the Go code under
// /root/reference/internal/raft (Go toolchain absent here):
//   raft.go, logentry.go, inmemory.go, remote.go, readindex.go,
//   entryutils.go, peer.go, and the TestLogDB fixture of logdb_test.go.
// Every function cites the reference file:line it follows. Semantics are kept
// exactly: uint64 arithmetic (wrap-around included), same branch order, same
// panics (thrown as oracle::Panic). Two deliberate, documented substitutions:
//   * Go map iteration over remotes/observers is random; here std::map gives
//     ascending node-ID order (parity is defined per
//     (group, To, Type) modulo this order).
//   * random.LockGuardedRand (internal/utils/random/rand.go:43-61) is replaced
//     by an injectable per-raft source so tests can pin it, exactly as the
//     reference tests do with setRandomizedElectionTimeout.
#pragma once

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace oracle {

using u64 = uint64_t;
struct Entry;

// Observation hooks for the batch harness's escalation predicate (batch.cpp):
// they record what an item did (term lookups, resets, campaigns, snapshot
// paths, appends) and never change behaviour. One probe per harness thread.
struct Probe {
  virtual ~Probe() {}
  virtual void lookup(u64 index) = 0;                          // a term()/entries() read inside [firstIndex-1, lastIndex]
  virtual void merged(const std::vector<Entry>& es) = 0;      // inMemory.merge
  virtual void resetCalled() = 0;                              // raft.reset
  virtual void campaignCalled() = 0;                           // raft.campaign
  virtual void replicateError() = 0;                           // makeReplicateMessage failed (InstallSnapshot path)
  virtual void replicateRange(u64 next, u64 last) = 0;         // makeReplicateMessage(next) with lastIndex last
  virtual void readIndexAdd(size_t queued, bool dup) = 0;      // readIndex.addRequest
};
inline thread_local Probe* g_probe = nullptr;

struct Panic : std::runtime_error {
  explicit Panic(const std::string& s) : std::runtime_error(s) {}
};

[[noreturn]] inline void panicf(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
inline void panicf(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  throw Panic(buf);
}

// raftpb/raft.pb.go:26-50
enum MessageType : uint32_t {
  LocalTick = 0, Election = 1, LeaderHeartbeat = 2, ConfigChangeEvent = 3,
  NoOP = 4, Ping = 5, Pong = 6, Propose = 7, SnapshotStatus = 8,
  Unreachable = 9, CheckQuorum = 10, BatchedReadIndex = 11, Replicate = 12,
  ReplicateResp = 13, RequestVote = 14, RequestVoteResp = 15,
  InstallSnapshot = 16, Heartbeat = 17, HeartbeatResp = 18, ReadIndex = 19,
  ReadIndexResp = 20, Quiesce = 21, SnapshotReceived = 22,
  LeaderTransfer = 23, TimeoutNow = 24,
};
constexpr u64 numMessageTypes = 25;  // raft.go:48

// raftpb/raft.pb.go:131-132
enum EntryType : uint32_t { ApplicationEntry = 0, ConfigChangeEntry = 1 };

// raftpb/raft.pb.go:414-423 (fields the step path reads; Cmd kept by length
// plus optional bytes so SizeUpperLimit is exact)
struct Entry {
  u64 Term = 0;
  u64 Index = 0;
  EntryType Type = ApplicationEntry;
  u64 Key = 0;
  std::vector<uint8_t> Cmd;
  // raftpb/raft_optimized.go:70-75
  int SizeUpperLimit() const { return 16 * 7 + 16 + (int)Cmd.size(); }
  bool operator==(const Entry& o) const {
    return Term == o.Term && Index == o.Index && Type == o.Type &&
           Key == o.Key && Cmd == o.Cmd;
  }
};

struct Membership {
  std::map<u64, std::string> Addresses;
  std::map<u64, std::string> Observers;
  std::map<u64, bool> Removed;
};

struct Snapshot {
  u64 Index = 0;
  u64 Term = 0;
  Membership membership;
};
inline bool IsEmptySnapshot(const Snapshot& s) { return s.Index == 0; }  // raftpb/raft.go:113

struct State {  // raftpb State
  u64 Term = 0, Vote = 0, Commit = 0;
};
inline bool IsStateEqual(const State& a, const State& b) {  // raftpb/raft.go:118-124
  return a.Term == b.Term && a.Vote == b.Vote && a.Commit == b.Commit;
}
inline bool IsEmptyState(const State& s) { return IsStateEqual(s, State{}); }

// raftpb/raft.go:38-41
struct SystemCtx {
  u64 Low = 0, High = 0;
  bool operator==(const SystemCtx& o) const { return Low == o.Low && High == o.High; }
  bool operator!=(const SystemCtx& o) const { return !(*this == o); }
  bool operator<(const SystemCtx& o) const {
    return Low < o.Low || (Low == o.Low && High < o.High);
  }
};

// raftpb/raft.go:45-48
struct ReadyToRead {
  u64 Index = 0;
  SystemCtx ctx;
};

// raftpb/raft.pb.go:780-794
struct Message {
  MessageType Type = LocalTick;
  u64 To = 0, From = 0, ClusterId = 0, Term = 0, LogTerm = 0, LogIndex = 0,
      Commit = 0;
  bool Reject = false;
  u64 Hint = 0;
  std::vector<Entry> Entries;
  Snapshot snapshot;
  u64 HintHigh = 0;
};

// raftpb/raft.go:52-58
struct UpdateCommit {
  u64 AppliedTo = 0, StableLogTo = 0, StableLogTerm = 0, StableSnapshotTo = 0,
      ReadyToRead = 0;
};

enum class Err { None, Compacted, SnapshotOutOfDate, Unavailable };  // logentry.go:31-40

constexpr u64 noLimit = UINT64_MAX;  // raft.go:47
constexpr u64 NoLeader = 0, NoNode = 0;  // raft.go:44-46
// internal/settings/hard.go:102 and soft.go:236
constexpr u64 MaxProposalPayloadSize = 32ull * 1024 * 1024;
constexpr u64 MaxEntrySize = 2 * MaxProposalPayloadSize;
constexpr u64 maxEntriesToApplySize = MaxProposalPayloadSize * 2;  // logentry.go:27

inline u64 min_(u64 x, u64 y) { return x > y ? y : x; }  // entryutils.go:65-70
inline u64 max_(u64 x, u64 y) { return x > y ? x : y; }  // entryutils.go:72-77

// entryutils.go:21-29
inline int countConfigChange(const std::vector<Entry>& es) {
  int c = 0;
  for (auto& e : es)
    if (e.Type == ConfigChangeEntry) c++;
  return c;
}

// entryutils.go:36-48
inline void checkEntriesToAppend(const std::vector<Entry>& ents,
                                 const std::vector<Entry>& toAppend) {
  if (ents.empty() || toAppend.empty()) return;
  if (ents.back().Index + 1 != toAppend[0].Index)
    panicf("found a hole, last %llu, first to append %llu",
           (unsigned long long)ents.back().Index,
           (unsigned long long)toAppend[0].Index);
  if (ents.back().Term > toAppend[0].Term)
    panicf("term value not expected, %llu vs %llu",
           (unsigned long long)ents.back().Term,
           (unsigned long long)toAppend[0].Term);
}

// entryutils.go:50-63
inline std::vector<Entry> limitSize(const std::vector<Entry>& ents, u64 limit) {
  if (ents.empty()) return ents;
  u64 total = (u64)ents[0].SizeUpperLimit();
  size_t inc;
  for (inc = 1; inc < ents.size(); inc++) {
    total += (u64)ents[inc].SizeUpperLimit();
    if (total > limit) break;
  }
  return std::vector<Entry>(ents.begin(), ents.begin() + inc);
}

inline std::vector<Entry> slice(const std::vector<Entry>& v, u64 lo, u64 hi) {
  if (lo > hi || hi > v.size()) panicf("slice bounds out of range [%llu:%llu] len %zu",
                                       (unsigned long long)lo, (unsigned long long)hi, v.size());
  return std::vector<Entry>(v.begin() + lo, v.begin() + hi);
}

// logentry.go:46-74 (read-only view of the persistent log)
struct ILogDB {
  virtual ~ILogDB() = default;
  virtual std::pair<u64, u64> GetRange() = 0;
  virtual State NodeState(Membership* m) = 0;
  virtual void SetState(const State& s) = 0;
  virtual Err CreateSnapshot(const Snapshot& ss) = 0;
  virtual Err ApplySnapshot(const Snapshot& ss) = 0;
  virtual u64 Term(u64 index, Err* err) = 0;
  virtual std::vector<Entry> Entries(u64 low, u64 high, u64 maxSize, Err* err) = 0;
  virtual Snapshot GetSnapshot() = 0;
  virtual Err Compact(u64 index) = 0;
  virtual Err Append(std::vector<Entry> entries) = 0;
};

// internal/raft/logdb_test.go:25-177 (TestLogDB, the reference's in-memory
// ILogDB fixture; also the shape of internal/logdb/logreader.go:131-166)
struct TestLogDB : ILogDB {
  std::vector<Entry> entries;
  u64 markerIndex = 0, markerTerm = 0;
  Snapshot snapshot;
  State state;

  std::pair<u64, u64> GetRange() override { return {firstIndex(), lastIndex()}; }
  u64 firstIndex() const { return markerIndex + 1; }
  u64 lastIndex() const { return markerIndex + (u64)entries.size(); }
  State NodeState(Membership* m) override {
    if (m) *m = snapshot.membership;
    return state;
  }
  void SetState(const State& s) override { state = s; }
  Snapshot GetSnapshot() override { return snapshot; }
  Err ApplySnapshot(const Snapshot& ss) override {  // :48-57
    if (snapshot.Index >= ss.Index) return Err::SnapshotOutOfDate;
    snapshot = ss;
    markerIndex = ss.Index;
    markerTerm = ss.Term;
    entries.clear();
    return Err::None;
  }
  Err CreateSnapshot(const Snapshot& ss) override {  // :59-65
    if (snapshot.Index >= ss.Index) return Err::SnapshotOutOfDate;
    snapshot = ss;
    return Err::None;
  }
  u64 Term(u64 index, Err* err) override {  // :99-112
    *err = Err::None;
    if (index == markerIndex) return markerTerm;
    auto ents = Entries(index, index + 1, UINT64_MAX, err);
    if (*err != Err::None) return 0;
    if (ents.empty()) return 0;
    return ents[0].Term;
  }
  Err Append(std::vector<Entry> es) override {  // :114-134
    if (es.empty()) return Err::None;
    u64 first = firstIndex();
    if (markerIndex + (u64)es.size() < first) return Err::None;
    if (first > es[0].Index) es = slice(es, first - es[0].Index, es.size());
    u64 offset = es[0].Index - markerIndex;
    if ((u64)entries.size() + 1 > offset) {
      entries = slice(entries, 0, offset - 1);
    } else if ((u64)entries.size() + 1 < offset) {
      panicf("found a hole last index %llu, first incoming index %llu",
             (unsigned long long)lastIndex(), (unsigned long long)es[0].Index);
    }
    entries.insert(entries.end(), es.begin(), es.end());
    return Err::None;
  }
  std::vector<Entry> Entries(u64 low, u64 high, u64 maxSize, Err* err) override {  // :136-150
    *err = Err::None;
    if (low <= markerIndex) { *err = Err::Compacted; return {}; }
    if (high > lastIndex() + 1) { *err = Err::Unavailable; return {}; }
    if (entries.empty()) { *err = Err::Unavailable; return {}; }
    auto ents = slice(entries, low - markerIndex - 1, high - markerIndex - 1);
    return limitSize(ents, maxSize);
  }
  Err Compact(u64 index) override {  // :152-177
    if (index <= markerIndex) return Err::Compacted;
    if (index > lastIndex()) return Err::Unavailable;
    if (entries.empty()) return Err::Unavailable;
    Err e;
    u64 term = Term(index, &e);
    if (e != Err::None) return e;
    u64 cut = index - markerIndex;
    entries = slice(entries, cut, entries.size());
    markerIndex = index;
    markerTerm = term;
    return Err::None;
  }
};

// inmemory.go:27-184
struct inMemory {
  std::unique_ptr<Snapshot> snapshot;
  std::vector<Entry> entries;
  u64 markerIndex = 0;
  u64 savedTo = 0;

  inMemory() = default;
  explicit inMemory(u64 lastIndex) : markerIndex(lastIndex + 1), savedTo(lastIndex) {}  // :36-41
  inMemory(const inMemory& o)
      : snapshot(o.snapshot ? new Snapshot(*o.snapshot) : nullptr),
        entries(o.entries), markerIndex(o.markerIndex), savedTo(o.savedTo) {}
  inMemory& operator=(const inMemory& o) {
    snapshot.reset(o.snapshot ? new Snapshot(*o.snapshot) : nullptr);
    entries = o.entries;
    markerIndex = o.markerIndex;
    savedTo = o.savedTo;
    return *this;
  }

  void checkMarkerIndex() const {  // :43-50
    if (!entries.empty() && entries[0].Index != markerIndex)
      panicf("marker index %llu, first index %llu", (unsigned long long)markerIndex,
             (unsigned long long)entries[0].Index);
  }
  std::vector<Entry> getEntries(u64 low, u64 high) const {  // :52-62
    u64 upperBound = markerIndex + (u64)entries.size();
    if (low > high || low < markerIndex)
      panicf("invalid low value %llu, high %llu, marker index %llu", (unsigned long long)low,
             (unsigned long long)high, (unsigned long long)markerIndex);
    if (high > upperBound)
      panicf("invalid high value %llu, upperBound %llu", (unsigned long long)high,
             (unsigned long long)upperBound);
    return slice(entries, low - markerIndex, high - markerIndex);
  }
  bool getSnapshotIndex(u64* idx) const {  // :64-69
    if (snapshot) { *idx = snapshot->Index; return true; }
    *idx = 0;
    return false;
  }
  bool getLastIndex(u64* idx) const {  // :71-76
    if (!entries.empty()) { *idx = entries.back().Index; return true; }
    return getSnapshotIndex(idx);
  }
  bool getTerm(u64 index, u64* t) const {  // :78-90
    *t = 0;
    if (index < markerIndex) {
      u64 idx;
      if (getSnapshotIndex(&idx) && idx == index) { *t = snapshot->Term; return true; }
      return false;
    }
    u64 lastIndex;
    bool ok = getLastIndex(&lastIndex);
    if (ok && index <= lastIndex) { *t = entries.at(index - markerIndex).Term; return true; }
    return false;
  }
  void commitUpdate(const UpdateCommit& cu) {  // :92-99
    if (cu.StableLogTo > 0) savedLogTo(cu.StableLogTo, cu.StableLogTerm);
    if (cu.StableSnapshotTo > 0) savedSnapshotTo(cu.StableSnapshotTo);
  }
  std::vector<Entry> entriesToSave() const {  // :101-108
    u64 idx = savedTo + 1;
    if (idx - markerIndex > (u64)entries.size()) return {};
    return slice(entries, idx - markerIndex, entries.size());
  }
  void savedLogTo(u64 index, u64 term) {  // :110-122
    if (index < markerIndex) return;
    if (entries.empty()) return;
    if (index > entries.back().Index || term != entries.at(index - markerIndex).Term) return;
    savedTo = index;
  }
  void appliedLogTo(u64 index) {  // :124-139
    if (index < markerIndex) return;
    if (entries.empty()) return;
    if (index > entries.back().Index) return;
    u64 newMarkerIndex = index;
    entries = slice(entries, newMarkerIndex - markerIndex, entries.size());
    markerIndex = newMarkerIndex;
    // resizeEntrySlice (:149-155) only re-allocates capacity.
    checkMarkerIndex();
  }
  void savedSnapshotTo(u64 index) {  // :141-147
    u64 idx;
    bool ok = getSnapshotIndex(&idx);
    if (ok && idx == index) snapshot.reset();
  }
  void merge(const std::vector<Entry>& ents) {  // :157-177
    if (g_probe) g_probe->merged(ents);
    u64 firstNewIndex = ents[0].Index;
    if (firstNewIndex == markerIndex + (u64)entries.size()) {
      checkEntriesToAppend(entries, ents);
      entries.insert(entries.end(), ents.begin(), ents.end());
    } else if (firstNewIndex <= markerIndex) {
      markerIndex = firstNewIndex;
      entries = ents;
      savedTo = firstNewIndex - 1;
    } else {
      auto existing = getEntries(markerIndex, firstNewIndex);
      checkEntriesToAppend(existing, ents);
      std::vector<Entry> n;
      n.reserve(existing.size() + ents.size());
      n.insert(n.end(), existing.begin(), existing.end());
      n.insert(n.end(), ents.begin(), ents.end());
      entries.swap(n);
      savedTo = min_(savedTo, firstNewIndex - 1);
    }
    checkMarkerIndex();
  }
  void restore(const Snapshot& ss) {  // :179-184
    snapshot.reset(new Snapshot(ss));
    markerIndex = ss.Index + 1;
    entries.clear();
    savedTo = ss.Index;
  }
};

// logentry.go:79-381
struct entryLog {
  ILogDB* logdb;
  inMemory inmem;
  u64 committed = 0;
  u64 applied = 0;
  std::function<void(u64)> onTryAppend;  // observation hook for the batch harness (no effect)

  // A struct literal &entryLog{logdb: db} as several reference tests build it
  // (e.g. raft_etcd_test.go:1916-1919): all other fields zero.
  entryLog(ILogDB* db, u64 inmemMarker) : logdb(db) { inmem.markerIndex = inmemMarker; }
  explicit entryLog(ILogDB* db) : logdb(db) {  // :86-95
    auto r = db->GetRange();
    inmem = inMemory(r.second);
    committed = r.first - 1;
    applied = r.first - 1;
  }
  u64 firstIndex() const {  // :97-104
    u64 index;
    if (inmem.getSnapshotIndex(&index)) return index + 1;
    return logdb->GetRange().first;
  }
  u64 lastIndex() const {  // :106-113
    u64 index;
    if (inmem.getLastIndex(&index)) return index;
    return logdb->GetRange().second;
  }
  std::pair<u64, u64> termEntryRange() const { return {firstIndex() - 1, lastIndex()}; }  // :115-124
  bool entryRange(u64* f, u64* l) const {  // :126-131
    if (inmem.snapshot && inmem.entries.empty()) return false;
    *f = firstIndex();
    *l = lastIndex();
    return true;
  }
  u64 lastTerm() const {  // :133-139
    Err e;
    u64 t = term(lastIndex(), &e);
    if (e != Err::None) panicf("lastTerm error");
    return t;
  }
  u64 term(u64 index, Err* err) const {  // :141-157
    *err = Err::None;
    auto r = termEntryRange();
    if (index < r.first || index > r.second) return 0;
    if (g_probe) g_probe->lookup(index);
    u64 t;
    if (inmem.getTerm(index, &t)) return t;
    Err e;
    t = logdb->Term(index, &e);
    if (e != Err::None && e != Err::Compacted && e != Err::Unavailable) panicf("logdb term error");
    if (e == Err::None) return t;
    *err = e;
    return 0;
  }
  Err checkBound(u64 low, u64 high) const {  // :159-174
    if (low > high) panicf("input low %llu > high %llu", (unsigned long long)low, (unsigned long long)high);
    u64 first, last;
    if (!entryRange(&first, &last)) return Err::Compacted;
    if (low < first) return Err::Compacted;
    if (high > last + 1)
      panicf("requested range [%llu,%llu) is out of bound [%llu,%llu]", (unsigned long long)low,
             (unsigned long long)high, (unsigned long long)first, (unsigned long long)last);
    return Err::None;
  }
  std::vector<Entry> getEntriesFromLogDB(u64 low, u64 high, u64 maxSize, bool* checkInMem,
                                         Err* err) const {  // :176-193
    *err = Err::None;
    if (low >= inmem.markerIndex) { *checkInMem = true; return {}; }
    u64 upperBound = min_(high, inmem.markerIndex);
    Err e;
    auto ents = logdb->Entries(low, upperBound, maxSize, &e);
    if (e == Err::Compacted) { *checkInMem = false; *err = e; return {}; }
    if (e != Err::None) panicf("logdb entries error %d", (int)e);
    if ((u64)ents.size() > upperBound - low) panicf("uint64(len(ents)) > upperBound-low");
    *checkInMem = (u64)ents.size() == upperBound - low;
    return ents;
  }
  std::vector<Entry> getEntriesFromInMem(std::vector<Entry> ents, u64 low, u64 high) const {  // :195-210
    if (high <= inmem.markerIndex) return ents;
    u64 lowerBound = max_(low, inmem.markerIndex);
    auto im = inmem.getEntries(lowerBound, high);
    if (!im.empty()) {
      if (!ents.empty()) {
        checkEntriesToAppend(ents, im);
        ents.insert(ents.end(), im.begin(), im.end());
        return ents;
      }
      return im;
    }
    return ents;
  }
  std::vector<Entry> getEntries(u64 low, u64 high, u64 maxSize, Err* err) const {  // :212-229
    *err = checkBound(low, high);
    if (*err != Err::None) return {};
    if (low == high) return {};
    if (g_probe) g_probe->lookup(low);
    bool checkInMem;
    auto ents = getEntriesFromLogDB(low, high, maxSize, &checkInMem, err);
    if (*err != Err::None) return {};
    if (!checkInMem) return ents;
    return limitSize(getEntriesFromInMem(ents, low, high), maxSize);
  }
  std::vector<Entry> entries(u64 start, u64 maxSize, Err* err) const {  // :231-236
    *err = Err::None;
    if (start > lastIndex()) return {};
    return getEntries(start, lastIndex() + 1, maxSize, err);
  }
  Snapshot snapshot() const {  // :238-243
    if (inmem.snapshot) return *inmem.snapshot;
    return logdb->GetSnapshot();
  }
  u64 firstNotAppliedIndex() const { return max_(applied + 1, firstIndex()); }  // :245-247
  u64 toApplyIndexLimit() const { return committed + 1; }  // :249-251
  bool hasEntriesToApply() const { return toApplyIndexLimit() > firstNotAppliedIndex(); }  // :253-255
  bool hasMoreEntriesToApply(u64 appliedTo) const { return committed > appliedTo; }  // :257-259
  std::vector<Entry> getEntriesToApply(u64 limit) const {  // :265-275
    if (hasEntriesToApply()) {
      Err e;
      auto ents = getEntries(firstNotAppliedIndex(), toApplyIndexLimit(), limit, &e);
      if (e != Err::None) panicf("getEntriesToApply error");
      return ents;
    }
    return {};
  }
  std::vector<Entry> entriesToApply() const { return getEntriesToApply(maxEntriesToApplySize); }  // :261-263
  std::vector<Entry> entriesToSave() const { return inmem.entriesToSave(); }  // :277-279
  bool tryAppend(u64 index, const std::vector<Entry>& ents) {  // :281-292
    u64 conflictIndex = getConflictIndex(ents);
    if (conflictIndex != 0) {
      if (conflictIndex <= committed)
        panicf("entry %llu conflicts with committed entry, committed %llu",
               (unsigned long long)conflictIndex, (unsigned long long)committed);
      if (onTryAppend) onTryAppend(conflictIndex);
      append(slice(ents, conflictIndex - index - 1, ents.size()));
      return true;
    }
    return false;
  }
  void append(const std::vector<Entry>& es) {  // :294-303
    if (es.empty()) return;
    if (es[0].Index <= committed)
      panicf("committed entries being changed, committed %llu, first idx %llu",
             (unsigned long long)committed, (unsigned long long)es[0].Index);
    inmem.merge(es);
  }
  u64 getConflictIndex(const std::vector<Entry>& es) const {  // :305-312
    for (auto& e : es)
      if (!matchTerm(e.Index, e.Term)) return e.Index;
    return 0;
  }
  void commitTo(u64 index) {  // :314-323
    if (index <= committed) return;
    if (index > lastIndex())
      panicf("invalid commitTo index %llu, lastIndex() %llu", (unsigned long long)index,
             (unsigned long long)lastIndex());
    committed = index;
  }
  void commitUpdate(const UpdateCommit& cu) {  // :325-335
    inmem.commitUpdate(cu);
    if (cu.AppliedTo > 0) {
      if (cu.AppliedTo < applied || cu.AppliedTo > committed)
        panicf("invalid applyto %llu, current applied %llu, committed %llu",
               (unsigned long long)cu.AppliedTo, (unsigned long long)applied,
               (unsigned long long)committed);
      applied = cu.AppliedTo;
      inmem.appliedLogTo(cu.AppliedTo);
    }
  }
  bool matchTerm(u64 index, u64 t) const {  // :337-343
    Err e;
    u64 lt = term(index, &e);
    if (e != Err::None) return false;
    return lt == t;
  }
  bool upToDate(u64 index, u64 t) const {  // :345-357
    Err e;
    u64 lastT = term(lastIndex(), &e);
    if (e != Err::None) panicf("failed to get the last term");
    if (t >= lastT) {
      if (t > lastT) return true;
      return index >= lastIndex();
    }
    return false;
  }
  bool tryCommit(u64 index, u64 t) {  // :359-374
    if (index <= committed) return false;
    Err e;
    u64 lterm = term(index, &e);
    if (e == Err::Compacted) lterm = 0;
    else if (e != Err::None) panicf("tryCommit term error");
    if (index > committed && lterm == t) {
      commitTo(index);
      return true;
    }
    return false;
  }
  void restore(const Snapshot& s) {  // :376-381
    inmem.restore(s);
    committed = s.Index;
    applied = s.Index;
  }
};

// remote.go:27-183
enum remoteStateType : u64 { remoteRetry = 0, remoteWait = 1, remoteReplicate = 2, remoteSnapshot = 3 };

struct remote {
  u64 match = 0, next = 0, snapshotIndex = 0;
  remoteStateType state = remoteRetry;
  bool active = false;

  void reset() { snapshotIndex = 0; }  // :61-63
  void becomeRetry() {  // :65-73
    if (state == remoteSnapshot) next = max_(match + 1, snapshotIndex + 1);
    else next = match + 1;
    reset();
    state = remoteRetry;
  }
  void retryToWait() { if (state == remoteRetry) state = remoteWait; }  // :75-79
  void waitToRetry() { if (state == remoteWait) state = remoteRetry; }  // :81-85
  void becomeWait() { becomeRetry(); retryToWait(); }  // :87-90
  void becomeReplicate() { next = match + 1; reset(); state = remoteReplicate; }  // :92-96
  void becomeSnapshot(u64 index) { reset(); snapshotIndex = index; state = remoteSnapshot; }  // :98-102
  void clearPendingSnapshot() { snapshotIndex = 0; }  // :104-106
  bool tryUpdate(u64 index) {  // :108-118
    if (next < index + 1) next = index + 1;
    if (match < index) { waitToRetry(); match = index; return true; }
    return false;
  }
  void progress(u64 lastIndex) {  // :120-128
    if (state == remoteReplicate) next = lastIndex + 1;
    else if (state == remoteRetry) retryToWait();
    else panicf("unexpected remote state");
  }
  void respondedTo() {  // :130-138
    if (state == remoteRetry) becomeReplicate();
    else if (state == remoteSnapshot) {
      if (match >= snapshotIndex) becomeRetry();
    }
  }
  bool decreaseTo(u64 rejected, u64 last) {  // :140-156
    if (state == remoteReplicate) {
      if (rejected <= match) return false;
      next = match + 1;
      return true;
    }
    if (next - 1 != rejected) return false;
    waitToRetry();
    next = max_(1, min_(rejected, last + 1));
    return true;
  }
  bool isPaused() const {  // :158-171
    switch (state) {
      case remoteRetry: return false;
      case remoteWait: return true;
      case remoteReplicate: return false;
      case remoteSnapshot: return true;
    }
    panicf("unexpected remote state");
  }
  bool isActive() const { return active; }
  void setActive() { active = true; }
  void setNotActive() { active = false; }
};

// readindex.go:21-116
struct readStatus {
  u64 index = 0, from = 0;
  SystemCtx ctx;
  std::map<u64, bool> confirmed;
};

struct readIndex {
  std::map<SystemCtx, std::shared_ptr<readStatus>> pending;
  std::vector<SystemCtx> queue;

  void addRequest(u64 index, SystemCtx ctx, u64 from) {  // :43-67
    if (g_probe) g_probe->readIndexAdd(queue.size(), pending.count(ctx) != 0);
    if (pending.count(ctx)) return;
    if (!queue.empty()) {
      auto it = pending.find(peepCtx());
      if (it == pending.end()) panicf("inconsistent pending and queue");
      if (index < it->second->index)
        panicf("index moved backward in readIndex, %llu:%llu", (unsigned long long)index,
               (unsigned long long)it->second->index);
    }
    queue.push_back(ctx);
    auto s = std::make_shared<readStatus>();
    s->index = index;
    s->from = from;
    s->ctx = ctx;
    pending[ctx] = s;
  }
  bool hasPendingRequest() const { return !queue.empty(); }  // :69-71
  SystemCtx peepCtx() const { return queue.back(); }  // :73-75
  std::vector<std::shared_ptr<readStatus>> confirm(SystemCtx ctx, u64 from, int quorum) {  // :77-116
    auto it = pending.find(ctx);
    if (it == pending.end()) return {};
    auto p = it->second;
    p->confirmed[from] = true;
    if ((int)p->confirmed.size() + 1 < quorum) return {};
    size_t done = 0;
    std::vector<std::shared_ptr<readStatus>> cs;
    for (auto& pctx : queue) {
      done++;
      auto sit = pending.find(pctx);
      if (sit == pending.end()) panicf("inconsistent pending and queue content");
      auto s = sit->second;
      cs.push_back(s);
      if (pctx == ctx) {
        for (auto& v : cs) {
          if (v->index > s->index) panicf("v.index > s.index is unexpected");
          v->index = s->index;
        }
        queue.erase(queue.begin(), queue.begin() + done);
        for (auto& v : cs) pending.erase(v->ctx);
        if (queue.size() != pending.size()) panicf("inconsistent length");
        return cs;
      }
    }
    return {};
  }
};

// config/config.go:46-88 (fields used by the raft core)
struct Config {
  u64 NodeID = 0, ClusterID = 0;
  bool IsObserver = false, CheckQuorum = false, Quiesce = false;
  u64 ElectionRTT = 0, HeartbeatRTT = 0;
  // config/config.go:92-109
  void Validate() const {
    if (NodeID <= 0) panicf("invalid NodeID, it must be >= 1");
    if (HeartbeatRTT <= 0) panicf("HeartbeatRTT must be > 0");
    if (ElectionRTT <= 0) panicf("ElectionRTT must be > 0");
    if (ElectionRTT <= 2 * HeartbeatRTT) panicf("invalid election rtt");
  }
};

enum RaftState : u64 { follower = 0, candidate = 1, leader = 2, observer = 3, numStates = 4 };  // raft.go:58-66

inline bool isLocalMessageType(MessageType t) {  // entryutils.go:86-94
  return t == Election || t == LeaderHeartbeat || t == Unreachable || t == SnapshotStatus ||
         t == CheckQuorum || t == LocalTick || t == BatchedReadIndex;
}
inline bool isResponseMessageType(MessageType t) {  // entryutils.go:96-104
  return t == ReplicateResp || t == RequestVoteResp || t == HeartbeatResp || t == ReadIndexResp ||
         t == Unreachable || t == SnapshotStatus || t == LeaderTransfer;
}
inline bool isRequestMessage(MessageType t) { return t == Propose || t == ReadIndex; }  // raft.go:982-984
inline bool isLeaderMessage(MessageType t) {  // raft.go:986-989
  return t == Replicate || t == InstallSnapshot || t == Heartbeat || t == TimeoutNow ||
         t == ReadIndexResp;
}

// default randomness: splitmix64 stream (stand-in for internal/utils/random)
struct SplitMix64 {
  u64 s;
  explicit SplitMix64(u64 seed) : s(seed) {}
  u64 operator()() {
    u64 z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
};

// raft.go:124-154
struct raft {
  using handlerFunc = void (raft::*)(const Message&);
  u64 applied = 0, nodeID = 0, clusterID = 0, term = 0, vote = 0;
  std::unique_ptr<entryLog> log;
  std::map<u64, remote> remotes;
  std::map<u64, remote> observers;
  RaftState state = follower;
  std::map<u64, bool> votes;
  std::vector<Message> msgs;
  u64 leaderID = 0, leaderTransferTarget = 0;
  bool isLeaderTransferTarget = false, pendingConfigChange = false;
  readIndex readIdx;
  std::vector<ReadyToRead> readyToRead;
  bool checkQuorum = false;
  u64 tickCount = 0, electionTick = 0, heartbeatTick = 0, heartbeatTimeout = 0,
      electionTimeout = 0, randomizedElectionTimeout = 0;
  std::vector<u64> matched;
  std::function<bool()> hasNotAppliedConfigChange;  // test hook, raft.go:152
  std::function<void(u64)> recordLeader;            // raft.go:153
  std::function<u64()> rng;                         // random.LockGuardedRand
  handlerFunc handlers[numStates][numMessageTypes] = {};

  // raft.go:156-201
  raft(const Config& c, ILogDB* logdb, std::function<u64()> rand = nullptr) {
    c.Validate();
    if (!logdb) panicf("logdb is nil");
    rng = rand ? rand : std::function<u64()>(SplitMix64(c.NodeID * 1000003ull + c.ClusterID));
    clusterID = c.ClusterID;
    nodeID = c.NodeID;
    leaderID = NoLeader;
    log.reset(new entryLog(logdb));
    electionTimeout = c.ElectionRTT;
    heartbeatTimeout = c.HeartbeatRTT;
    checkQuorum = c.CheckQuorum;
    Membership members;
    State st = logdb->NodeState(&members);
    for (auto& kv : members.Addresses) { remote r; r.next = 1; remotes[kv.first] = r; }
    for (auto& kv : members.Observers) { remote r; r.next = 1; observers[kv.first] = r; }
    resetMatchValueArray();
    if (!IsEmptyState(st)) loadState(st);
    if (c.IsObserver) {
      state = observer;
      becomeObserver(term, NoLeader);
    } else {
      becomeFollower(term, NoLeader);
    }
    initializeHandlerMap();
    checkHandlerMap();
  }

  void setTestPeers(const std::vector<u64>& peers) {  // :203-209
    if (remotes.empty())
      for (u64 p : peers) { remote r; r.next = 1; remotes[p] = r; }
  }
  void setApplied(u64 a) { applied = a; }
  u64 getApplied() const { return applied; }
  void resetMatchValueArray() { matched.assign(remotes.size(), 0); }  // :219-221
  bool isObserver() const { return state == observer; }
  void setLeaderID(u64 id) {  // :239-244
    leaderID = id;
    if (recordLeader) recordLeader(leaderID);
  }
  bool leaderTransfering() const { return leaderTransferTarget != NoNode && state == leader; }  // :246-248
  void abortLeaderTransfer() { leaderTransferTarget = NoNode; }
  int quorum() const { return (int)remotes.size() / 2 + 1; }  // :254-256
  bool isSingleNodeQuorum() const { return quorum() == 1; }
  bool leaderHasQuorum() {  // :262-271
    int c = 0;
    for (auto& kv : remotes) {
      if (kv.first == nodeID || kv.second.isActive()) {
        c++;
        kv.second.setNotActive();
      }
    }
    return c >= quorum();
  }
  std::vector<u64> nodes() const {  // :273-283
    std::vector<u64> n;
    for (auto& kv : remotes) n.push_back(kv.first);
    for (auto& kv : observers) n.push_back(kv.first);
    std::sort(n.begin(), n.end());
    return n;
  }
  State raftState() const { return State{term, vote, log->committed}; }  // :285-291
  void loadState(const State& st) {  // :293-301
    if (st.Commit < log->committed || st.Commit > log->lastIndex())
      panicf("got out of range state, st.commit %llu, range[%llu,%llu]",
             (unsigned long long)st.Commit, (unsigned long long)log->committed,
             (unsigned long long)log->lastIndex());
    log->committed = st.Commit;
    term = st.Term;
    vote = st.Vote;
  }
  bool restore(const Snapshot& ss) {  // :303-325
    if (ss.Index <= log->committed) return false;
    if (!isObserver()) {
      for (auto& kv : ss.membership.Observers)
        if (kv.first == nodeID) panicf("converting to observer");
    }
    if (log->matchTerm(ss.Index, ss.Term)) {
      log->commitTo(ss.Index);
      return false;
    }
    log->restore(ss);
    return true;
  }
  void restoreRemotes(const Snapshot& ss) {  // :327-355
    remotes.clear();
    for (auto& kv : ss.membership.Addresses) {
      u64 id = kv.first;
      if (observers.count(id)) becomeFollower(term, leaderID);
      u64 match = 0, next = log->lastIndex() + 1;
      if (id == nodeID) match = next - 1;
      setRemote(id, match, next);
    }
    observers.clear();
    for (auto& kv : ss.membership.Observers) {
      u64 id = kv.first;
      u64 match = 0, next = log->lastIndex() + 1;
      if (id == nodeID) match = next - 1;
      setObserver(id, match, next);
    }
    resetMatchValueArray();
  }

  // tick related functions, raft.go:361-438
  bool timeForElection() const { return electionTick >= randomizedElectionTimeout; }
  bool timeForHearbeat() const { return heartbeatTick >= heartbeatTimeout; }
  bool timeForCheckQuorum() const { return electionTick >= electionTimeout; }
  bool timeToAbortLeaderTransfer() const { return leaderTransfering() && electionTick >= electionTimeout; }
  void tick() {  // :377-384
    tickCount++;
    if (state == leader) leaderTick();
    else nonLeaderTick();
  }
  void nonLeaderTick() {  // :386-401
    if (state == leader) panicf("noleader tick called on leader node");
    electionTick++;
    if (isObserver()) return;
    if (!selfRemoved() && timeForElection()) {
      electionTick = 0;
      Message m; m.From = nodeID; m.Type = Election;
      Handle(m);
    }
  }
  void leaderTick() {  // :403-429
    if (state != leader) panicf("leaderTick called on a non-leader node");
    electionTick++;
    bool abortLT = timeToAbortLeaderTransfer();
    if (timeForCheckQuorum()) {
      electionTick = 0;
      if (checkQuorum) { Message m; m.From = nodeID; m.Type = CheckQuorum; Handle(m); }
    }
    if (abortLT) abortLeaderTransfer();
    heartbeatTick++;
    if (timeForHearbeat()) {
      heartbeatTick = 0;
      Message m; m.From = nodeID; m.Type = LeaderHeartbeat;
      Handle(m);
    }
  }
  void quiescedTick() { electionTick++; }  // :431-433
  void setRandomizedElectionTimeout() {  // :435-438
    if (electionTimeout == 0) panicf("runtime error: integer divide by zero");  // Go's % by zero
    u64 randTime = rng() % electionTimeout;
    randomizedElectionTimeout = electionTimeout + randTime;
  }

  // send and broadcast, raft.go:444-594
  Message finalizeMessageTerm(Message m) const {  // :444-455
    if (m.Term == 0 && m.Type == RequestVote) panicf("sending RequestVote with 0 term");
    if (m.Term > 0 && m.Type != RequestVote) panicf("term unexpectedly set for message type %u", m.Type);
    if (!isRequestMessage(m.Type)) m.Term = term;
    return m;
  }
  void send(Message m) {  // :457-461
    m.From = nodeID;
    m = finalizeMessageTerm(m);
    msgs.push_back(std::move(m));
  }
  u64 makeInstallSnapshotMessage(u64 to, Message* m) {  // :463-472
    m->To = to;
    m->Type = InstallSnapshot;
    Snapshot s = log->snapshot();
    if (IsEmptySnapshot(s)) panicf("got an empty snapshot");
    m->snapshot = s;
    return s.Index;
  }
  Message makeReplicateMessage(u64 to, u64 next, u64 maxSize, Err* err) {  // :474-498
    if (g_probe) g_probe->replicateRange(next, log->lastIndex());
    u64 t = log->term(next - 1, err);
    if (*err != Err::None) return Message{};
    auto ents = log->entries(next, maxSize, err);
    if (*err != Err::None) return Message{};
    if (!ents.empty() && ents.back().Index != next - 1 + (u64)ents.size())
      panicf("expected last index in Replicate");
    Message m;
    m.To = to;
    m.Type = Replicate;
    m.LogIndex = next - 1;
    m.LogTerm = t;
    m.Entries = std::move(ents);
    m.Commit = log->committed;
    return m;
  }
  remote* findRemote(u64 id) {
    auto it = remotes.find(id);
    if (it != remotes.end()) return &it->second;
    auto ot = observers.find(id);
    if (ot != observers.end()) return &ot->second;
    return nullptr;
  }
  u64 maxEntrySize = MaxEntrySize;  // settings.Soft.MaxEntrySize
  void sendReplicateMessage(u64 to) {  // :500-532
    remote* rp = findRemote(to);
    if (!rp) panicf("failed to get the remote instance");
    if (rp->isPaused()) return;
    Err err;
    Message m = makeReplicateMessage(to, rp->next, maxEntrySize, &err);
    if (err != Err::None) {
      if (g_probe) g_probe->replicateError();
      if (!rp->isActive()) return;
      u64 index = makeInstallSnapshotMessage(to, &m);
      rp->becomeSnapshot(index);
    } else {
      if (!m.Entries.empty()) rp->progress(m.Entries.back().Index);
    }
    send(std::move(m));
  }
  void broadcastReplicateMessage() {  // :534-546
    for (auto& kv : remotes)
      if (kv.first != nodeID) sendReplicateMessage(kv.first);
    for (auto& kv : observers) {
      if (kv.first == nodeID) panicf("observer is trying to broadcast Replicate msg");
      sendReplicateMessage(kv.first);
    }
  }
  void sendHeartbeatMessage(u64 to, SystemCtx hint, bool toObserver) {  // :548-564
    u64 match = toObserver ? observers.at(to).match : remotes.at(to).match;
    u64 commit = min_(match, log->committed);
    Message m;
    m.To = to;
    m.Type = Heartbeat;
    m.Commit = commit;
    m.Hint = hint.Low;
    m.HintHigh = hint.High;
    send(std::move(m));
  }
  void broadcastHeartbeatMessage() {  // :566-573
    if (readIdx.hasPendingRequest()) broadcastHeartbeatMessageWithHint(readIdx.peepCtx());
    else broadcastHeartbeatMessageWithHint(SystemCtx{});
  }
  void broadcastHeartbeatMessageWithHint(SystemCtx ctx) {  // :575-587
    SystemCtx zeroCtx;
    for (auto& kv : remotes)
      if (kv.first != nodeID) sendHeartbeatMessage(kv.first, ctx, false);
    if (ctx == zeroCtx)
      for (auto& kv : observers) sendHeartbeatMessage(kv.first, zeroCtx, true);
  }
  void sendTimeoutNowMessage(u64 target) {  // :589-594
    Message m;
    m.Type = TimeoutNow;
    m.To = target;
    send(std::move(m));
  }

  // log append and commit, raft.go:600-654
  void sortMatchValues() {  // :600-623
    if (matched.size() == 3) {
      if (matched[0] > matched[1]) std::swap(matched[0], matched[1]);
      if (matched[1] > matched[2]) std::swap(matched[1], matched[2]);
      if (matched[0] > matched[1]) std::swap(matched[0], matched[1]);
    } else {
      std::sort(matched.begin(), matched.end());
    }
  }
  bool tryCommit() {  // :625-641
    if (remotes.size() != matched.size()) resetMatchValueArray();
    size_t idx = 0;
    for (auto& kv : remotes) matched[idx++] = kv.second.match;
    sortMatchValues();
    u64 q = matched[remotes.size() - (size_t)quorum()];
    return log->tryCommit(q, term);
  }
  void appendEntries(std::vector<Entry>& es) {  // :643-654
    u64 lastIndex = log->lastIndex();
    for (size_t i = 0; i < es.size(); i++) {
      es[i].Term = term;
      es[i].Index = lastIndex + 1 + (u64)i;
    }
    log->append(es);
    remotes.at(nodeID).tryUpdate(log->lastIndex());
    if (isSingleNodeQuorum()) tryCommit();
  }

  // state transitions, raft.go:660-753
  void becomeObserver(u64 t, u64 leaderID_) {  // :660-667
    if (state != observer) panicf("transitioning to observer state from non-observer");
    reset(t);
    setLeaderID(leaderID_);
  }
  void becomeFollower(u64 t, u64 leaderID_) {  // :669-674
    state = follower;
    reset(t);
    setLeaderID(leaderID_);
  }
  void becomeCandidate() {  // :676-687
    if (state == leader) panicf("transitioning to candidate state from leader");
    if (state == observer) panicf("observer is becoming candidate");
    state = candidate;
    reset(term + 1);
    vote = nodeID;
  }
  void becomeLeader() {  // :689-702
    if (state == follower) panicf("transitioning to leader state from follower");
    if (state == observer) panicf("observer is become leader");
    state = leader;
    reset(term);
    setLeaderID(nodeID);
    preLeaderPromotionHandleConfigChange();
    std::vector<Entry> es(1);
    appendEntries(es);
  }
  void reset(u64 t) {  // :704-720
    if (g_probe) g_probe->resetCalled();
    if (term != t) {
      term = t;
      vote = NoLeader;
    }
    setLeaderID(NoLeader);
    votes.clear();
    electionTick = 0;
    heartbeatTick = 0;
    setRandomizedElectionTimeout();
    readIdx = readIndex{};
    clearPendingConfigChange();
    abortLeaderTransfer();
    resetRemotes();
    resetObservers();
    resetMatchValueArray();
  }
  void preLeaderPromotionHandleConfigChange() {  // :722-731
    int n = getPendingConfigChangeCount();
    if (n > 1) panicf("multiple uncommitted config change entries");
    else if (n == 1) setPendingConfigChange();
  }
  void resetRemotes() {  // :733-742
    for (auto& kv : remotes) {
      remote r;
      r.next = log->lastIndex() + 1;
      if (kv.first == nodeID) r.match = log->lastIndex();
      kv.second = r;
    }
  }
  void resetObservers() {  // :744-753
    for (auto& kv : observers) {
      remote r;
      r.next = log->lastIndex() + 1;
      if (kv.first == nodeID) r.match = log->lastIndex();
      kv.second = r;
    }
  }

  // election, raft.go:759-807
  int handleVoteResp(u64 from, bool rejected) {
    int votedFor = 0;
    if (!votes.count(from)) votes[from] = !rejected;
    for (auto& kv : votes)
      if (kv.second) votedFor++;
    return votedFor;
  }
  void campaign() {  // :779-807
    if (g_probe) g_probe->campaignCalled();
    becomeCandidate();
    u64 t = term;
    handleVoteResp(nodeID, false);
    if (isSingleNodeQuorum()) {
      becomeLeader();
      return;
    }
    u64 hint = 0;
    if (isLeaderTransferTarget) {
      hint = nodeID;
      isLeaderTransferTarget = false;
    }
    for (auto& kv : remotes) {
      if (kv.first == nodeID) continue;
      Message m;
      m.Term = t;
      m.To = kv.first;
      m.Type = RequestVote;
      m.LogIndex = log->lastIndex();
      m.LogTerm = log->lastTerm();
      m.Hint = hint;
      send(std::move(m));
    }
  }

  // membership, raft.go:813-917
  bool selfRemoved() const {  // :813-820
    if (state == observer) return observers.find(nodeID) == observers.end();
    return remotes.find(nodeID) == remotes.end();
  }
  void addNode(u64 id) {  // :822-839
    clearPendingConfigChange();
    if (remotes.count(id)) return;
    auto it = observers.find(id);
    if (it != observers.end()) {
      remote rp = it->second;
      deleteObserver(id);
      remotes[id] = rp;
      if (id == nodeID) becomeFollower(term, leaderID);
    } else {
      setRemote(id, 0, log->lastIndex() + 1);
    }
  }
  void addObserver(u64 id) {  // :841-847
    clearPendingConfigChange();
    if (observers.count(id)) return;
    setObserver(id, 0, log->lastIndex() + 1);
  }
  void removeNode(u64 id) {  // :849-861
    deleteRemote(id);
    deleteObserver(id);
    clearPendingConfigChange();
    if (leaderTransfering() && leaderTransferTarget == id) abortLeaderTransfer();
    if (!remotes.empty())
      if (tryCommit()) broadcastReplicateMessage();
  }
  void deleteRemote(u64 id) { remotes.erase(id); resetMatchValueArray(); }
  void deleteObserver(u64 id) { observers.erase(id); }
  void setRemote(u64 id, u64 match, u64 next) {  // :872-880
    remote r;
    r.next = next;
    r.match = match;
    remotes[id] = r;
    resetMatchValueArray();
  }
  void setObserver(u64 id, u64 match, u64 next) {  // :882-889
    remote r;
    r.next = next;
    r.match = match;
    observers[id] = r;
  }
  void setPendingConfigChange() { pendingConfigChange = true; }
  bool hasPendingConfigChange() const { return pendingConfigChange; }
  void clearPendingConfigChange() { pendingConfigChange = false; }
  int getPendingConfigChangeCount() {  // :903-917
    u64 idx = log->committed + 1;
    int count = 0;
    for (;;) {
      Err e;
      auto ents = log->entries(idx, maxEntriesToApplySize, &e);
      if (e != Err::None) panicf("failed to get entries");
      if (ents.empty()) return count;
      count += countConfigChange(ents);
      idx = ents.back().Index + 1;
    }
  }

  // handlers, raft.go:923-976
  void handleHeartbeatMessage(const Message& m) {  // :923-931
    log->commitTo(m.Commit);
    Message r;
    r.To = m.From;
    r.Type = HeartbeatResp;
    r.Hint = m.Hint;
    r.HintHigh = m.HintHigh;
    send(std::move(r));
  }
  void handleInstallSnapshotMessage(const Message& m) {  // :933-951
    Message resp;
    resp.To = m.From;
    resp.Type = ReplicateResp;
    if (restore(m.snapshot)) resp.LogIndex = log->lastIndex();
    else resp.LogIndex = log->committed;
    send(std::move(resp));
  }
  void handleReplicateMessage(const Message& m) {  // :953-976
    Message resp;
    resp.To = m.From;
    resp.Type = ReplicateResp;
    if (m.LogIndex < log->committed) {
      resp.LogIndex = log->committed;
      send(std::move(resp));
      return;
    }
    if (log->matchTerm(m.LogIndex, m.LogTerm)) {
      log->tryAppend(m.LogIndex, m.Entries);
      u64 lastIdx = m.LogIndex + (u64)m.Entries.size();
      log->commitTo(min_(lastIdx, m.Commit));
      resp.LogIndex = lastIdx;
    } else {
      resp.Reject = true;
      resp.LogIndex = m.LogIndex;
      resp.Hint = log->lastIndex();
    }
    send(std::move(resp));
  }

  // step, raft.go:991-1053
  bool dropRequestVoteFromHighTermNode(const Message& m) const {  // :991-1009
    if (m.Type != RequestVote || !checkQuorum || m.Term <= term) return false;
    if (m.Hint == m.From) return false;
    if (leaderID != NoLeader && electionTick < electionTimeout) return true;
    return false;
  }
  bool onMessageTermNotMatched(const Message& m) {  // :1014-1044
    if (m.Term == 0 || m.Term == term) return false;
    if (dropRequestVoteFromHighTermNode(m)) return true;
    if (m.Term > term) {
      u64 lid = NoLeader;
      if (isLeaderMessage(m.Type)) lid = m.From;
      if (isObserver()) becomeObserver(m.Term, lid);
      else becomeFollower(m.Term, lid);
    } else if (m.Term < term) {
      if (isLeaderMessage(m.Type) && checkQuorum) {
        Message r;
        r.To = m.From;
        r.Type = NoOP;
        send(std::move(r));
      }
      return true;
    }
    return false;
  }
  void Handle(const Message& m) {  // :1046-1053
    if (!onMessageTermNotMatched(m)) {
      doubleCheckTermMatched(m.Term);
      defaultHandle(m);
    }
  }
  bool hasConfigChangeToApply() const {  // :1055-1061
    if (hasNotAppliedConfigChange) return hasNotAppliedConfigChange();
    return log->committed > getApplied();
  }
  bool canGrantVote(const Message& m) const {  // :1063-1067
    return vote == NoNode || vote == m.From || m.Term > term;
  }
  void handleNodeElection(const Message&) {  // :1073-1086
    if (state != leader) {
      if (hasConfigChangeToApply()) return;
      campaign();
    }
  }
  void handleNodeRequestVote(const Message& m) {  // :1088-1107
    Message resp;
    resp.To = m.From;
    resp.Type = RequestVoteResp;
    bool canGrant = canGrantVote(m);
    bool isUpToDate = log->upToDate(m.LogIndex, m.LogTerm);
    if (canGrant && isUpToDate) {
      electionTick = 0;
      vote = m.From;
    } else {
      resp.Reject = true;
    }
    send(std::move(resp));
  }
  void handleLeaderLeaderHeartbeat(const Message&) { broadcastHeartbeatMessage(); }  // :1113-1115
  void handleLeaderCheckQuorum(const Message&) {  // :1117-1123
    if (!leaderHasQuorum()) becomeFollower(term, NoLeader);
  }
  void handleLeaderPropose(const Message& mm) {  // :1125-1146
    Message m = mm;
    if (selfRemoved()) return;
    if (leaderTransfering()) return;
    for (auto& e : m.Entries) {
      if (e.Type == ConfigChangeEntry) {
        if (hasPendingConfigChange()) e = Entry{};
        setPendingConfigChange();
      }
    }
    appendEntries(m.Entries);
    broadcastReplicateMessage();
  }
  bool hasCommittedEntryAtCurrentTerm() const {  // :1148-1157
    if (term == 0) panicf("not suppose to reach here");
    Err e;
    u64 lastCommittedTerm = log->term(log->committed, &e);
    if (e != Err::None && e != Err::Compacted) panicf("hasCommittedEntryAtCurrentTerm");
    return lastCommittedTerm == term;
  }
  void clearReadyToRead() { readyToRead.clear(); }
  void addReadyToRead(u64 index, SystemCtx ctx) { readyToRead.push_back(ReadyToRead{index, ctx}); }
  void handleLeaderReadIndex(const Message& m) {  // :1171-1203
    // selfRemoved() only logs here (:1172-1174)
    SystemCtx ctx{m.Hint, m.HintHigh};
    if (!isSingleNodeQuorum()) {
      if (!hasCommittedEntryAtCurrentTerm()) return;
      readIdx.addRequest(log->committed, ctx, m.From);
      broadcastHeartbeatMessageWithHint(ctx);
    } else {
      addReadyToRead(log->committed, ctx);
      if (m.From != nodeID && observers.count(m.From)) {
        Message r;
        r.To = m.From;
        r.Type = ReadIndexResp;
        r.LogIndex = log->committed;
        r.Hint = m.Hint;
        r.HintHigh = m.HintHigh;
        r.Commit = m.Commit;
        send(std::move(r));
      }
    }
  }
  void handleLeaderReplicateResp(const Message& m, remote* rp) {  // :1205-1227
    rp->setActive();
    if (!m.Reject) {
      bool paused = rp->isPaused();
      if (rp->tryUpdate(m.LogIndex)) {
        rp->respondedTo();
        if (tryCommit()) broadcastReplicateMessage();
        else if (paused) sendReplicateMessage(m.From);
        if (leaderTransfering() && m.From == leaderTransferTarget && log->lastIndex() == rp->match)
          sendTimeoutNowMessage(leaderTransferTarget);
      }
    } else {
      if (rp->decreaseTo(m.LogIndex, m.Hint)) {
        enterRetryState(rp);
        sendReplicateMessage(m.From);
      }
    }
  }
  void handleLeaderHeartbeatResp(const Message& m, remote* rp) {  // :1229-1240
    rp->setActive();
    rp->waitToRetry();
    if (rp->match < log->lastIndex()) sendReplicateMessage(m.From);
    if (m.Hint != 0) handleReadIndexLeaderConfirmation(m);
  }
  void handleLeaderLeaderTransfer(const Message& m, remote* rp) {  // :1242-1262
    u64 target = m.Hint;
    if (target == NoNode) panicf("leader transfer target not set");
    if (leaderTransfering()) return;
    if (nodeID == target) return;
    leaderTransferTarget = target;
    electionTick = 0;
    if (rp->match == log->lastIndex()) sendTimeoutNowMessage(target);
  }
  void handleReadIndexLeaderConfirmation(const Message& m) {  // :1264-1284
    SystemCtx ctx{m.Hint, m.HintHigh};
    auto ris = readIdx.confirm(ctx, m.From, quorum());
    for (auto& s : ris) {
      if (s->from == NoNode || s->from == nodeID) {
        addReadyToRead(s->index, s->ctx);
      } else {
        Message r;
        r.To = s->from;
        r.Type = ReadIndexResp;
        r.LogIndex = s->index;
        r.Hint = m.Hint;
        r.HintHigh = m.HintHigh;
        send(std::move(r));
      }
    }
  }
  void handleLeaderSnapshotStatus(const Message& m, remote* rp) {  // :1286-1299
    if (rp->state != remoteSnapshot) return;
    if (m.Reject) rp->clearPendingSnapshot();
    rp->becomeWait();
  }
  void handleLeaderUnreachable(const Message&, remote* rp) { enterRetryState(rp); }  // :1301-1305
  void enterRetryState(remote* rp) {  // :1307-1311
    if (rp->state == remoteReplicate) rp->becomeRetry();
  }
  // observer handlers, :1318-1340
  void handleObserverReplicate(const Message& m) { handleFollowerReplicate(m); }
  void handleObserverHeartbeat(const Message& m) { handleFollowerHeartbeat(m); }
  void handleObserverSnapshot(const Message& m) { handleFollowerInstallSnapshot(m); }
  void handleObserverPropose(const Message& m) { handleFollowerPropose(m); }
  void handleObserverReadIndex(const Message& m) { handleFollowerReadIndex(m); }
  void handleObserverReadIndexResp(const Message& m) { handleFollowerReadIndexResp(m); }
  // follower handlers, :1346-1417
  void handleFollowerPropose(const Message& mm) {
    if (leaderID == NoLeader) return;
    Message m = mm;
    m.To = leaderID;
    send(std::move(m));
  }
  void handleFollowerReplicate(const Message& m) {
    electionTick = 0;
    setLeaderID(m.From);
    handleReplicateMessage(m);
  }
  void handleFollowerHeartbeat(const Message& m) {
    electionTick = 0;
    setLeaderID(m.From);
    handleHeartbeatMessage(m);
  }
  void handleFollowerReadIndex(const Message& mm) {
    if (leaderID == NoLeader) return;
    Message m = mm;
    m.To = leaderID;
    send(std::move(m));
  }
  void handleFollowerLeaderTransfer(const Message& mm) {
    if (leaderID == NoLeader) return;
    Message m = mm;
    m.To = leaderID;
    send(std::move(m));
  }
  void handleFollowerReadIndexResp(const Message& m) {
    SystemCtx ctx{m.Hint, m.HintHigh};
    electionTick = 0;
    setLeaderID(m.From);
    addReadyToRead(m.LogIndex, ctx);
  }
  void handleFollowerInstallSnapshot(const Message& m) {
    electionTick = 0;
    setLeaderID(m.From);
    handleInstallSnapshotMessage(m);
  }
  void handleFollowerTimeoutNow(const Message&) {
    electionTick = randomizedElectionTimeout;
    isLeaderTransferTarget = true;
    tick();
    if (isLeaderTransferTarget) isLeaderTransferTarget = false;
  }
  // candidate handlers, :1423-1464
  void doubleCheckTermMatched(u64 msgTerm) const {
    if (msgTerm != 0 && term != msgTerm) panicf("mismatched term found");
  }
  void handleCandidatePropose(const Message&) {}
  void handleCandidateReplicate(const Message& m) {
    becomeFollower(term, m.From);
    handleReplicateMessage(m);
  }
  void handleCandidateInstallSnapshot(const Message& m) {
    becomeFollower(term, m.From);
    handleInstallSnapshotMessage(m);
  }
  void handleCandidateHeartbeat(const Message& m) {
    becomeFollower(term, m.From);
    handleHeartbeatMessage(m);
  }
  void handleCandidateRequestVoteResp(const Message& m) {
    if (observers.count(m.From)) return;
    int count = handleVoteResp(m.From, m.Reject);
    if (count == quorum()) {
      becomeLeader();
      broadcastReplicateMessage();
    } else if ((int)votes.size() - count == quorum()) {
      becomeFollower(term, NoLeader);
    }
  }
  // lw wrappers, :1466-1479
  void lwReplicateResp(const Message& m) { lw(m, &raft::handleLeaderReplicateResp); }
  void lwHeartbeatResp(const Message& m) { lw(m, &raft::handleLeaderHeartbeatResp); }
  void lwSnapshotStatus(const Message& m) { lw(m, &raft::handleLeaderSnapshotStatus); }
  void lwUnreachable(const Message& m) { lw(m, &raft::handleLeaderUnreachable); }
  void lwLeaderTransfer(const Message& m) { lw(m, &raft::handleLeaderLeaderTransfer); }
  void lw(const Message& m, void (raft::*f)(const Message&, remote*)) {
    auto it = remotes.find(m.From);
    if (it != remotes.end()) { (this->*f)(m, &it->second); return; }
    auto ot = observers.find(m.From);
    if (ot != observers.end()) { (this->*f)(m, &ot->second); return; }
  }
  void defaultHandle(const Message& m) {  // :1481-1486
    handlerFunc f = handlers[state][m.Type];
    if (f) (this->*f)(m);
  }
  void initializeHandlerMap() {  // :1488-1527
    handlers[candidate][Heartbeat] = &raft::handleCandidateHeartbeat;
    handlers[candidate][Propose] = &raft::handleCandidatePropose;
    handlers[candidate][Replicate] = &raft::handleCandidateReplicate;
    handlers[candidate][InstallSnapshot] = &raft::handleCandidateInstallSnapshot;
    handlers[candidate][RequestVoteResp] = &raft::handleCandidateRequestVoteResp;
    handlers[candidate][Election] = &raft::handleNodeElection;
    handlers[candidate][RequestVote] = &raft::handleNodeRequestVote;
    handlers[follower][Propose] = &raft::handleFollowerPropose;
    handlers[follower][Replicate] = &raft::handleFollowerReplicate;
    handlers[follower][Heartbeat] = &raft::handleFollowerHeartbeat;
    handlers[follower][ReadIndex] = &raft::handleFollowerReadIndex;
    handlers[follower][LeaderTransfer] = &raft::handleFollowerLeaderTransfer;
    handlers[follower][ReadIndexResp] = &raft::handleFollowerReadIndexResp;
    handlers[follower][InstallSnapshot] = &raft::handleFollowerInstallSnapshot;
    handlers[follower][Election] = &raft::handleNodeElection;
    handlers[follower][RequestVote] = &raft::handleNodeRequestVote;
    handlers[follower][TimeoutNow] = &raft::handleFollowerTimeoutNow;
    handlers[leader][LeaderHeartbeat] = &raft::handleLeaderLeaderHeartbeat;
    handlers[leader][CheckQuorum] = &raft::handleLeaderCheckQuorum;
    handlers[leader][Propose] = &raft::handleLeaderPropose;
    handlers[leader][ReadIndex] = &raft::handleLeaderReadIndex;
    handlers[leader][ReplicateResp] = &raft::lwReplicateResp;
    handlers[leader][HeartbeatResp] = &raft::lwHeartbeatResp;
    handlers[leader][SnapshotStatus] = &raft::lwSnapshotStatus;
    handlers[leader][Unreachable] = &raft::lwUnreachable;
    handlers[leader][LeaderTransfer] = &raft::lwLeaderTransfer;
    handlers[leader][Election] = &raft::handleNodeElection;
    handlers[leader][RequestVote] = &raft::handleNodeRequestVote;
    handlers[observer][Heartbeat] = &raft::handleObserverHeartbeat;
    handlers[observer][Replicate] = &raft::handleObserverReplicate;
    handlers[observer][InstallSnapshot] = &raft::handleObserverSnapshot;
    handlers[observer][Propose] = &raft::handleObserverPropose;
    handlers[observer][ReadIndex] = &raft::handleObserverReadIndex;
    handlers[observer][ReadIndexResp] = &raft::handleObserverReadIndexResp;
  }
  void checkHandlerMap() const {  // :1529-1559
    const std::pair<RaftState, MessageType> checks[] = {
        {leader, Heartbeat},          {leader, Replicate},         {leader, InstallSnapshot},
        {leader, ReadIndexResp},      {follower, ReplicateResp},   {follower, HeartbeatResp},
        {follower, SnapshotStatus},   {follower, Unreachable},     {candidate, ReplicateResp},
        {candidate, HeartbeatResp},   {candidate, SnapshotStatus}, {candidate, Unreachable},
        {observer, Election},         {observer, RequestVote},     {observer, RequestVoteResp},
        {observer, ReplicateResp},    {observer, HeartbeatResp},
    };
    for (auto& c : checks)
      if (handlers[c.first][c.second]) panicf("unexpected msg handler");
  }

  std::vector<Message> readMessages() {  // raft_etcd_test.go:118-123
    std::vector<Message> m;
    m.swap(msgs);
    return m;
  }
  // raft_etcd_test.go:48-55
  bool testOnlyHasConfigChangeToApply() const {
    auto ents = log->getEntriesToApply(noLimit);
    if (log->committed > log->applied && !ents.empty()) return countConfigChange(ents) > 0;
    return false;
  }
};

// peer.go:33-337 — the Peer API the host (node.go) drives.
struct Peer {
  u64 leaderID = 0;
  std::unique_ptr<raft> r;
  State prevState;

  void Tick() { r->tick(); }                 // :104-107
  void QuiescedTick() { r->quiescedTick(); }  // :109-112
  void ProposeEntries(std::vector<Entry> ents) {  // :126-134
    Message m;
    m.Type = Propose;
    m.From = r->nodeID;
    m.Entries = std::move(ents);
    r->Handle(m);
  }
  void ReadIndex(SystemCtx ctx) {  // :262-269
    Message m;
    m.Type = oracle::ReadIndex;
    m.Hint = ctx.Low;
    m.HintHigh = ctx.High;
    r->Handle(m);
  }
  void Handle(const Message& m) {  // :199-209
    if (isLocalMessageType(m.Type)) panicf("local message sent to Step");
    bool rok = r->remotes.count(m.From) > 0;
    bool ook = r->observers.count(m.From) > 0;
    if (rok || ook || !isResponseMessageType(m.Type)) r->Handle(m);
  }
  void ReportUnreachableNode(u64 nodeID) {  // :188-194
    Message m;
    m.Type = Unreachable;
    m.From = nodeID;
    r->Handle(m);
  }
  void ReportSnapshotStatus(u64 nodeID, bool reject) {  // :196-204
    Message m;
    m.Type = SnapshotStatus;
    m.From = nodeID;
    m.Reject = reject;
    r->Handle(m);
  }
  void RequestLeaderTransfer(u64 target) {  // :114-124
    Message m;
    m.Type = LeaderTransfer;
    m.To = r->nodeID;
    m.From = target;
    m.Hint = target;
    r->Handle(m);
  }
  void NotifyRaftLastApplied(u64 lastApplied) { r->setApplied(lastApplied); }  // :293-297
};

}  // namespace oracle
