// gr_fast.h — the lean steady-state lane of the step kernel.
//
// Most lanes of a pass are in one of two steady states:
//   leader:   ReplicateResp accepts at the current term, then ProposeEntries
//             (raft.go:1205-1227 handleLeaderReplicateResp, tryCommit
//             :625-641, broadcastReplicateMessage :534-546, handleLeaderPropose
//             :1125-1146);
//   follower: Replicate at the current term from one remote, appending at the
//             end of its log (raft.go:1359-1363, handleReplicateMessage
//             :953-976, logentry.go:281-312 tryAppend/getConflictIndex).
// fast_step<S> restates exactly that subset of the general lane (gr_lane.h,
// same field semantics, same message fields) with every remote slot a
// compile-time index, the term window reduced to its newest run, and all
// loads issued in three rounds before any store. Anything else — another
// message type, a term mismatch, a reject, a lookup below the newest run, a
// truncation, ticks, ReadIndex, more than two messages in a mailbox — returns
// false before the first state store; the general lane then steps the lane
// from its untouched state (message bodies this lane may have written to its
// out mailboxes are overwritten there, and their counts were never written).
#pragma once
#include "gr_cover.h"
#include "gr_layout.h"

namespace gr {

#define GF_HD __host__ __device__ inline __attribute__((always_inline))
// A condition outside the steady state clears `ok`; the lane keeps computing
// (branch-light, no early exits: keeps the exec-mask nesting shallow) and
// hands over at the end. Nothing but uncounted message bodies is stored
// before `ok` is checked.
// GF_BAIL re-reads `ok` after evaluating its condition: a condition that bails
// itself (below_newest inside term_of) must not be overwritten by the outer one.
#ifdef GR_BAIL_TRACE
// Diagnostic host build of the lane code only (tools/bail_trace.py): counts, per
// source line, the first steady-state condition that handed a lane over.
void gr_bail_trace(int line);
#define GF_BAIL(c) (ok = ok ? !((c) ? (gr_bail_trace(__LINE__), true) : false) && ok : false)
#else
#define GF_BAIL(c) (ok = ok ? !(c) && ok : false)
#endif

// Lane roles a lean-lane instance is built for (gr_kernels.h launches one
// kernel per role over the waves whose hint names it): FL_ANY steps leaders and
// followers; FL_LEADER and FL_FOLLOWER drop the other role's code (and its
// registers) and hand such a lane to the general lane.
constexpr int FL_ANY = 0, FL_LEADER = 1, FL_FOLLOWER = 2;

template <int S, int R = FL_ANY, int RM = RM_ANY>
struct FastLane {
  using Rw = Rows<S>;
  // RM: the route mode this instance is built for (gr_layout.h routes_of);
  // RT_LOOPBACK spaces have one chunk, so a mailbox address is plain arithmetic
  static constexpr bool kOneChunk = RM == RT_LOOPBACK;
  GF_HD Mailbox min_at(uint32_t g) const { return kp.in.template at<kOneChunk>(g); }
  GF_HD Mailbox mout_at(uint32_t g) const { return kp.out.template at<kOneChunk>(g); }
  static constexpr int MK = 2;  // messages per mailbox handled here
  // Leaders with input run here for up to 3 slots; wider groups' leaders take
  // the general lane (keeps this kernel's code and registers small for S = 5)
  static constexpr bool kLeaderPath = S <= 3 && R != FL_FOLLOWER;
  static constexpr bool kFollowerPath = R != FL_LEADER;
  static constexpr bool kSync = has_sync_bits(S);  // header sync bits (gr_layout.h)

  const StepParams& kp;
  const uint32_t i, p;
  // core
  uint64_t hdr = 0;  // the header word as loaded (gr_layout.h)
  uint32_t state = 0, self = 0, nruns = 0;
  uint64_t term = 0, committed = 0, committed0 = 0, hi = 0, hi0 = 0;
  uint64_t rsn = 0, rtn = 0;  // newest term run (start, term)
  uint64_t rsn0 = 0, rtn0 = 0;  // ... as loaded (moves one row down when a run is pushed)
  // run bits (gr_layout.h): with both set and the rows not loaded, rsn is
  // unknown but at most cload (committed as loaded) and rtn is term
  static constexpr bool kRuns = has_run_bits(S);
  bool rknown = true;
  uint64_t cload = 0;
  bool runs_out = false;  // both run bits set after the pass (the wave hint)
  // "x is below the newest run's start" when rsn is unknown is answered only for
  // x at or above cload (no); below it the lane hands over
  GF_HD bool below_newest(uint64_t x) {
    if (rknown) return x < rsn;
    GF_BAIL(x < cload);
    return false;
  }
  bool pushed = false;        // a run was appended this pass (row nruns-1)
  bool ok = true;             // still on the steady-state path
  // leader remotes
  uint64_t match[S], next[S];
  // per remote slot state (2 bits), active (1), kind (2): the header's rb
  // layout (gr_layout.h), one register instead of 3S
  uint64_t rbw = 0;
  GF_HD uint32_t rst(int j) const { return rb_state(rbw, (uint32_t)j); }
  GF_HD uint32_t ract(int j) const { return rb_active(rbw, (uint32_t)j); }
  GF_HD uint32_t rkind(int j) const { return rb_kind(rbw, (uint32_t)j); }
  GF_HD void set_rst(int j, uint32_t v) { rbw = rb_with(rbw, (uint32_t)j, 0, 2, v); }
  GF_HD void set_ract(int j, uint32_t v) { rbw = rb_with(rbw, (uint32_t)j, 2, 1, v); }
  uint32_t mdirty = 0;  // slots whose match/next changed
  uint32_t sdirty = 0;  // slots whose state/active byte changed
  uint32_t snapz = 0;
  uint32_t have_m = 0, have_n = 0;  // slots whose MATCH / NEXT row was loaded with the hint
  bool synced = false;              // after the pass: every member slot's next and own match in sync
  bool skipped = false;             // the lane is the other role instance's (step returned false)
  // emission
  uint32_t gout[S];
  uint32_t outc[S];
  uint32_t n1out = 0;    // leader: bit 8j + k = out Replicate k of slot j carries an entry
  uint32_t fullout = 0;  // leader: bit 8j + k = out Replicate k of slot j is a full record (not compact)
  const uint64_t max_entry;  // StepParams::max_entry_size, read once
  uint32_t rejout = 0;   // follower: bit k = out ReplicateResp k is a reject (not uniform: tags written)
  uint32_t nmo = 0, nmi = 0, nent = 0;
  uint32_t lslot_out = 0;  // F_LSLOT after the pass (the wave hint)
  bool had_input = false;   // messages or proposals this pass
  // results
  uint64_t append_from = 0;
  uint32_t prop_result = 0;

  GF_HD FastLane(const StepParams& k, uint32_t lane, uint32_t peer, uint64_t max_entry_size)
      : max_entry(max_entry_size), kp(k), i(lane), p(peer) {}

  GF_HD uint64_t& s64(uint32_t row) const { return kp.st.u64(row)[p]; }
  GF_HD uint8_t& s8(uint32_t row) const { return kp.st.u8(row)[p]; }

  // entryLog.term (logentry.go:141-157) when the answer is in the newest run.
  // The lane only runs with H_GE_LO (newest run start >= firstIndex-1), so
  // x >= rsn is inside [firstIndex-1, lastIndex]; anything below the newest
  // run (an older run, or below firstIndex-1) hands the lane over.
  GF_HD uint64_t term_of(uint64_t x) {
    if (x > hi) return 0;
    GF_BAIL(nruns == 0 || below_newest(x));
    return rtn;
  }
  // win_push (gr_lane.h) for one new run per pass onto a window of at most one
  // run: the right-aligned rows then move only the old newest run down one row
  // (a longer window would shift every run: the general lane does that).
  GF_HD void win_push(uint64_t start, uint64_t t) {
    if (nruns > 0 && rtn == t) return;
    GF_BAIL(pushed || nruns >= 2 || !rknown);  // moving the old newest run down needs its rows
    rsn = start;
    rtn = t;
    nruns++;
    pushed = true;
  }
  // raft.send (raft.go:457-461) of a Replicate into slot j, as Lane::emit writes
  // it: a compact Replicate (LogTerm = Term, at most one entry at Term) travels
  // in the hot fields only (a uniform mailbox when all are compact); any other
  // (a multi-entry catch-up, a LogTerm from the newest run's older term) also
  // writes its tag, term, entry count, LogTerm and run term.
  GF_HD void emit_replicate(int j, uint64_t log_index, uint64_t log_term, uint32_t n, uint64_t rt0) {
    GF_BAIL(gout[j] == NOPOS || outc[j] >= kp.out.depth);
    GF_BAIL(wide_term(term, log_term, n ? rt0 : 0, 0));  // GR_ESC_WIDE_TERM in the general lane
    uint32_t cd;
    GF_BAIL(!commit_delta(committed, log_index, &cd));  // a wide Commit: the general lane writes it
    if (!ok) return;
    const bool compact = log_term == term && (n == 0 || (n == 1 && rt0 == term));
    const Mailbox mb = mout_at(gout[j]);
    const uint32_t c = outc[j];
    n1out |= (n ? 1u : 0u) << (8 * j + c);  // MB_N1 bits: finish_out
    ntst(mb.u64(c, MF_LOG_INDEX), (uint64_t)(log_index));
    ntst(mb.t32(c, MT_CDELTA), (uint32_t)(cd));
    if (!compact) {
      fullout |= 1u << (8 * j + c);
      ntst(mb.tag(c), (uint16_t)(GR_REPLICATE | ((uint32_t)((n ? 1u : 0u) << MFL_RUNS_SHIFT) << 8)));
      ntst(mb.t32(c, MT_TERM), (uint32_t)term);
      ntst(mb.n(c), n);
      ntst(mb.t32(c, MT_LOG_TERM), (uint32_t)log_term);
      if (n) ntst(mb.t32(c, MT_RT0), (uint32_t)rt0);
    }
    outc[j] = c + 1;
    nmo++;
  }
  // ... and of a ReplicateResp into the mailbox at gpos (reject bits into rejout).
  GF_HD void emit_resp(uint32_t gpos, uint32_t* cnt, uint64_t log_index, bool reject, uint64_t hint) {
    GF_BAIL(gpos == NOPOS || *cnt >= kp.out.depth || *cnt >= kUniformMax);
    GF_BAIL(wide_term(term, 0, 0, 0));
    if (!ok) return;
    const Mailbox mb = mout_at(gpos);
    const uint32_t c = *cnt;
    rejout |= (reject ? 1u : 0u) << c;  // tags and terms: finish_out
    ntst(mb.u64(c, MF_LOG_INDEX), (uint64_t)(log_index));
    if (reject) ntst(mb.u64(c, MF_HINT), (uint64_t)(hint));
    *cnt = c + 1;
    nmo++;
  }

  // The count byte of out mailbox j, and the tags and terms its messages need:
  // a leader's compact Replicates (at most kUniformMax) and a follower's accepts
  // make a uniform mailbox (MB_UNIFORM, the term word, the entry bits); otherwise
  // every message gets its tag and term (a leader's compact ones as MFL_COMPACT
  // records, read_msg's form; its full records have theirs already).
  GF_HD void finish_out(int j, bool lead) {
    const uint32_t c = outc[j];
    uint32_t cb = c;
    if (c) {
      const Mailbox mb = mout_at(gout[j]);
      const uint32_t fo = (fullout >> (8 * j)) & 0xFFu, n1 = (n1out >> (8 * j)) & 0xFFu;
      if (lead ? (fo == 0 && c <= kUniformMax) : !rejout) {
        cb |= MB_UNIFORM | (lead ? 0u : (uint32_t)MB_RESP) | (lead ? (n1 & 7u) << MB_N1_SHIFT : 0u);
        ntst(mb.mterm(), (uint32_t)term);
      } else {
#pragma unroll
        for (uint32_t k = 0; k < (uint32_t)GR_C; ++k) {
          if (k < c && !(lead && ((fo >> k) & 1u))) {
            const uint32_t tg = lead ? GR_REPLICATE | ((uint32_t)(MFL_COMPACT | (((n1 >> k) & 1u)
                                                                                ? MFL_N1 | (1u << MFL_RUNS_SHIFT)
                                                                                : 0u)) << 8)
                                     : GR_REPLICATE_RESP | (((rejout >> k) & 1u) ? (uint32_t)MFL_REJECT << 8 : 0u);
            ntst(mb.tag(k), (uint16_t)tg);
            ntst(mb.t32(k, MT_TERM), (uint32_t)term);
          }
        }
      }
    }
    ntst(mout_at(gout[j]).cnt(), (uint8_t)cb);
  }

  // ------------------------------------------------------------- leader
  // raft.tryCommit + sortMatchValues + entryLog.tryCommit (raft.go:600-641,
  // logentry.go:359-374): order statistic of the voting match values by an
  // odd-even transposition network; non-voters sort to the end as +inf.
  GF_HD bool try_commit() {
    uint64_t m[S];
    int nv = 0;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const bool v = rkind(j) == GR_SLOT_VOTER;
      m[j] = v ? match[j] : ~0ull;
      nv += v;
    }
    GF_BAIL(nv == 0);
#pragma unroll
    for (int r = 0; r < S; ++r) {
#pragma unroll
      for (int x = (r & 1); x + 1 < S; x += 2) {
        const uint64_t a = m[x], b = m[x + 1];
        m[x] = a < b ? a : b;
        m[x + 1] = a < b ? b : a;
      }
    }
    const int qi = nv - (nv / 2 + 1);
    uint64_t q = m[0];
#pragma unroll
    for (int x = 1; x < S; ++x) q = (x == qi) ? m[x] : q;
    if (q <= committed) return false;
    const uint64_t lt = term_of(q);
    if (lt != term) return false;
    GF_BAIL(q > hi);  // commitTo panics (logentry.go:318-321)
    committed = q;
    return true;
  }
  // sendReplicateMessage / makeReplicateMessage (raft.go:474-532), one entry at most.
  GF_HD void send_replicate(int j) {
    if (rst(j) == GR_WAIT || rst(j) == GR_SNAPSHOT_ST) return;  // isPaused, remote.go:158-171
    const uint64_t nx = next[j];
    const uint64_t lt = term_of(nx - 1);
    uint32_t n = 0;
    if (nx <= hi) {
      // nx <= rsn covers entries in an older run and nx <= firstIndex-1
      // (InstallSnapshot path): with H_GE_LO, nx > rsn implies nx > firstIndex-1
      GF_BAIL(nruns == 0 || below_newest(nx - 1));  // nx <= rsn
      const uint64_t cnt = hi - nx + 1;  // entries nx..hi, all in the newest run
      // limitSize (entryutils.go:50-63) keeps all iff their sum fits (Lane::send_replicate)
      // (cnt > max / eub as cnt * eub > max: exact while both are below 2^32; a
      // bound of 4 GiB or more goes to the general lane)
      if (cnt > 1) {  // the entry-size bound row, loaded only for a lagging remote
        const uint64_t eub = ntld(s64(SR_ENTRY_UB));
        GF_BAIL(eub == 0 || (eub >> 32) != 0 || cnt > 0xFFFFFFFFull || cnt * eub > max_entry);
      }
      GF_BAIL(rst(j) != GR_REPLICATE_ST && rst(j) != GR_RETRY);
      n = (uint32_t)cnt;
      if (rst(j) == GR_REPLICATE_ST) {  // remote.progress, remote.go:120-128
        next[j] = hi + 1;
        mdirty |= 1u << j;
      } else {
        set_rst(j, GR_WAIT);
        sdirty |= 1u << j;
      }
    }
    emit_replicate(j, nx - 1, lt, n, rtn);
  }
  GF_HD void broadcast_kind(uint32_t ob) {
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const bool v = rkind(j) == GR_SLOT_VOTER && (uint32_t)j != self;
      const bool o = rkind(j) == GR_SLOT_OBSERVER;
      if (ob ? o : v) {
        GF_BAIL(ob && (uint32_t)j == self);
        send_replicate(j);
      }
    }
  }
  GF_HD void broadcast() {  // raft.go:534-546: voters (not self), then observers
    // one copy of send_replicate per slot: the voters / observers loop stays
    // rolled (code size: this is inlined at every message); S = 1 unrolls it
    // (rolled, its lane object does not stay in registers)
    if constexpr (S == 1) {
      broadcast_kind(0);
      broadcast_kind(1);
    } else {
#pragma unroll 1
      for (uint32_t ob = 0; ob < 2; ++ob) broadcast_kind(ob);
    }
  }
  // remote.tryUpdate (remote.go:108-118)
  GF_HD bool try_update(int j, uint64_t index) {
    if (next[j] < index + 1) {
      next[j] = index + 1;
      mdirty |= 1u << j;
    }
    if (match[j] < index) {
      if (rst(j) == GR_WAIT) {
        set_rst(j, GR_RETRY);
        sdirty |= 1u << j;
      }
      match[j] = index;
      mdirty |= 1u << j;
      return true;
    }
    return false;
  }
  // handleLeaderReplicateResp, accept path (raft.go:1205-1221); no leader transfer.
  GF_HD void replicate_resp(int j, uint64_t index) {
    if (!ract(j)) {
      set_ract(j, 1);
      sdirty |= 1u << j;
    }
    const bool paused = rst(j) == GR_WAIT || rst(j) == GR_SNAPSHOT_ST;
    if (!try_update(j, index)) return;
    GF_BAIL(rst(j) == GR_SNAPSHOT_ST);
    if (rst(j) == GR_RETRY) {  // respondedTo -> becomeReplicate (remote.go:92-96,130-138)
      next[j] = match[j] + 1;
      snapz |= 1u << j;
      set_rst(j, GR_REPLICATE_ST);
      mdirty |= 1u << j;
      sdirty |= 1u << j;
    }
    if (try_commit()) broadcast();
    else if (paused) send_replicate(j);
  }
  // handleLeaderPropose + appendEntries (raft.go:1125-1146, 643-654)
  GF_HD void propose(uint32_t np) {
    uint32_t sk = GR_SLOT_EMPTY;
#pragma unroll
    for (int j = 0; j < S; ++j) sk = ((uint32_t)j == self) ? rkind(j) : sk;
    if (sk != GR_SLOT_VOTER) {  // selfRemoved: dropped (raft.go:1126-1129)
      prop_result = GR_PROP_DROPPED;
      return;
    }
    GF_BAIL(nruns > 0 && rtn > term);  // checkEntriesToAppend would panic
    const uint64_t first = hi + 1;
    win_push(first, term);
    hi += np;
#pragma unroll
    for (int j = 0; j < S; ++j)
      if ((uint32_t)j == self) try_update(j, hi);
    int nv = 0;
#pragma unroll
    for (int j = 0; j < S; ++j) nv += rkind(j) == GR_SLOT_VOTER;
    if (nv / 2 + 1 == 1) try_commit();
    broadcast();
    prop_result = GR_PROP_APPENDED;
  }

  // ------------------------------------------------------------- step
  // `hint` (wave-uniform, gr_layout.h WH_*) says what the lane's wave was at the
  // end of the previous pass: all leaders, or all followers of one leader slot.
  // The loads that role needs are then issued with the header, in one round,
  // before the lane knows its state; a lane whose role differs from the hint
  // loads what it needs afterwards, so the hint never changes a result.
  // `take`: FL_ANY = step the lane whatever its role; FL_LEADER / FL_FOLLOWER =
  // step it only in that role (a leader / not a leader), else leave it untouched
  // with `skipped` set: the other role instance steps it (unhinted waves).
  GF_HD bool step(LaneStats* ls, uint32_t hint, int take = FL_ANY) {
    const bool hl = kLeaderPath && (hint & WH_ROLE) == WH_LEADER;
    const bool hf = (hint & WH_ROLE) == WH_FOLLOWER;
    const uint32_t hL = (hint >> WH_SLOT_SHIFT) & 7u;
    const bool hruns = kRuns && (hint & WH_RUNS);  // the wave's run bits were set: skip the run rows
    const uint32_t hself = (hint >> WH_SLOT_SHIFT) & 7u;  // leader hints: the self slot
    const bool hsync = kSync && hl && (hint & WH_SYNC);   // ... whose remote rows were in sync
    // ---- routes first: pure arithmetic, so no address of round 1 waits on a load
    uint32_t gin[S];
    routes_of<S, RM>(kp, i, gin, gout);
    // ---- round 1: core (one header word), the newest run (a fixed row), locals,
    //      mailbox counts, and the hinted role's loads
    hdr = ntld(s64(SR_HDR));
    term = ntld(s64(SR_TERM));
    committed = ntld(s64(SR_COMMITTED));
    hi = ntld(s64(SR_LAST_INDEX));
    if (!hruns) {
      rsn0 = ntld(s64(SR_RUN_START + GR_K - 1));  // meaningful when nruns > 0
      rtn0 = ntld(s64(SR_RUN_TERM + GR_K - 1));
    }
    const uint32_t lw = kp.has_locals ? ntld(kp.ln.u32(LR_LWORD)[i]) : 0u;  // packed locals (gr_layout.h)
#pragma unroll
    for (int j = 0; j < S; ++j) outc[j] = 0;
    // Mailboxes: the lean lane reads uniform ones only (MB_UNIFORM: every tag and
    // term implied by the count byte and the term word); any other hands over
    uint32_t cnt[S], cbs[S];
    uint32_t nonu = 0;  // in mailboxes holding messages without MB_UNIFORM
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const uint32_t b = gin[j] != NOPOS ? (uint32_t)ntld(min_at(gin[j]).cnt()) : 0u;
      cnt[j] = mb_n(b);
      cbs[j] = b;
      nonu |= (mb_n(b) && !(b & MB_UNIFORM)) ? (1u << j) : 0u;
    }
    // leader: the term word and LogIndexes of every in-mailbox (ReplicateResp accepts)
    uint32_t lmt[S];
    uint64_t lidx[S][MK];
    if (hl) {  // speculative: match/next (those a synced wave needs), the term word and LogIndexes
#pragma unroll
      for (int j = 0; j < S; ++j) {
        if (!hsync) {  // a synced wave's MATCH rows are all stale (H_MS, H_MP)
          match[j] = ntld(s64(Rw::MATCH + j));
          have_m |= 1u << j;
        }
        if (!hsync) {
          next[j] = ntld(s64(Rw::NEXT + j));
          have_n |= 1u << j;
        }
        lmt[j] = gin[j] != NOPOS ? ntld(min_at(gin[j]).mterm()) : 0u;
#pragma unroll
        for (int k = 0; k < MK; ++k) lidx[j][k] = gin[j] != NOPOS ? ntld(min_at(gin[j]).u64(k, MF_LOG_INDEX)) : 0;
      }
    }
    // follower: the term word, LogIndexes and Commit offsets of the one slot L that sent
    uint32_t fcd[MK];
    uint64_t fidx[MK];
    uint32_t fmt = 0;  // the sender's term word
#pragma unroll
    for (int k = 0; k < MK; ++k) {
      fidx[k] = 0;
      fcd[k] = 0;
    }
    uint32_t ghL = NOPOS;
    if (hf) {  // speculative: the hinted leader slot's term word and two compact Replicates
#pragma unroll
      for (int j = 0; j < S; ++j) ghL = ((uint32_t)j == hL) ? gin[j] : ghL;
      if (ghL != NOPOS) {
        const Mailbox mb = min_at(ghL);
        fmt = ntld(mb.mterm());
#pragma unroll
        for (int k = 0; k < MK; ++k) {
          fidx[k] = ntld(mb.u64(k, MF_LOG_INDEX));
          fcd[k] = ntld(mb.t32(k, MT_CDELTA));
        }
      }
    }
    state = h_state(hdr);
    self = h_self(hdr);
    nruns = h_nruns(hdr);
    const bool gelo = h_gelo(hdr);
    const uint32_t flags = h_flags(hdr);
    lslot_out = (flags & F_LSLOT) >> F_LSLOT_SHIFT;
    cload = committed;
    if (nruns) {
      if (hruns && kRuns && (hdr & H_RUN_MASK) == H_RUN_MASK) {
        rknown = false;  // rsn <= cload, rtn = term: the rows stay unread
        rtn = term;
      } else {
        if (hruns) {  // the hint misjudged this lane: its rows now
          rsn0 = ntld(s64(SR_RUN_START + GR_K - 1));
          rtn0 = ntld(s64(SR_RUN_TERM + GR_K - 1));
        }
        rsn = rsn0;
        rtn = rtn0;
      }
    }
    const bool leader = state == GR_LEADER;
    if ((take == FL_LEADER && !leader) || (take == FL_FOLLOWER && leader)) {
      skipped = true;
      return false;
    }
    const uint32_t np = lw & 0xFFFFu;
    const uint32_t nq = (lw & LW_OTHER) ? 0u : (lw >> LW_QT_SHIFT) & LW_QT_MAX;
    uint64_t etick = 0;
    if (nq) etick = ntld(s64(SR_ETICK));
    // ---- round 2 (only where the hint did not match): leader remotes and messages
    if (kLeaderPath && leader) {
      rbw = h_rb(hdr) & ((1ull << (5 * S)) - 1);
      // remote rows: stale ones (sync bits) from lastIndex, the rest loaded unless
      // the hint did. Every load of this round is issued before any value is used,
      // each at its row or, when not needed, at the header's line (loaded already),
      // and the values pass through keep_value: a branch around each load made one
      // round trip per slot (gr_layout.h keep_value).
      const uint64_t sb = kSync ? hdr : 0;
      uint64_t mv[S], nv[S];
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const bool ms = h_ms(sb) && (uint32_t)j == self, mp = h_mp(sb, (uint32_t)j) && (uint32_t)j != self;
        const bool lm = !ms && !mp && !((have_m >> j) & 1u), ln = !h_nx(sb, (uint32_t)j) && !((have_n >> j) & 1u);
        mv[j] = ntld(s64(lm ? (uint32_t)(Rw::MATCH + j) : (uint32_t)SR_HDR));
        nv[j] = ntld(s64(ln ? (uint32_t)(Rw::NEXT + j) : (uint32_t)SR_HDR));
      }
      uint32_t lmr[S];
      uint64_t lir[S][MK];
      if (!hl) {  // wave-uniform
#pragma unroll
        for (int j = 0; j < S; ++j) {
          lmr[j] = ntld(min_at(cnt[j] ? gin[j] : 0u).mterm());
#pragma unroll
          for (int k = 0; k < MK; ++k) {
            const bool ck = (uint32_t)k < cnt[j];
            lir[j][k] = ntld(min_at(ck ? gin[j] : 0u).u64(ck ? (uint32_t)k : 0u, MF_LOG_INDEX));
          }
        }
      }
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const bool ms = h_ms(sb) && (uint32_t)j == self, mp = h_mp(sb, (uint32_t)j) && (uint32_t)j != self;
        const uint64_t m = keep_value(mv[j]), n = keep_value(nv[j]);
        if (ms) match[j] = hi;
        else if (mp) match[j] = hi - 2;
        else if (!((have_m >> j) & 1u)) match[j] = m;
        if (h_nx(sb, (uint32_t)j)) next[j] = hi + 1;
        else if (!((have_n >> j) & 1u)) next[j] = n;
      }
      if (!hl) {
#pragma unroll
        for (int j = 0; j < S; ++j) {
          const uint32_t t = keep_value(lmr[j]);
          lmt[j] = cnt[j] ? t : 0u;
#pragma unroll
          for (int k = 0; k < MK; ++k) {
            const uint64_t v = keep_value(lir[j][k]);
            lidx[j][k] = (uint32_t)k < cnt[j] ? v : 0;
          }
        }
      }
    }
    if (kLeaderPath && leader) {
#pragma unroll
      for (int j = 0; j < S; ++j)  // a shared ack pair (MB_SHARED): message 1 = message 0 + 1
        if (mb_shared(cbs[j])) lidx[j][1] = lidx[j][0] + 1;
    }
    uint32_t L = 0, nsrc = 0, c = 0, gl = 0, go = NOPOS, cbL = 0;
    uint32_t fdrop = 0;  // follower: messages of uniform mailboxes at a lower term, dropped
    uint64_t rid = 0;
    if (kFollowerPath && !(kLeaderPath && leader)) {
      // the term word of every uniform mailbox with messages (the hinted one's is
      // loaded already): one at a lower term is dropped whole (raft.go:1014-1044),
      // unless it holds Replicates and checkQuorum asks for a NoOP reply
      // (one batch: address-selected loads, then keep_value, as the leader's round 2)
      uint32_t ft[S], ftr[S];
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const bool have = hf && (uint32_t)j == hL && ghL != NOPOS;
        const bool need = !have && cnt[j] && !((nonu >> j) & 1u);
        ftr[j] = ntld(min_at(need ? gin[j] : 0u).mterm());
      }
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const bool have = hf && (uint32_t)j == hL && ghL != NOPOS;
        const bool need = !have && cnt[j] && !((nonu >> j) & 1u);
        const uint32_t t = keep_value(ftr[j]);
        ft[j] = have ? fmt : need ? t : 0u;
      }
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const bool lower = cnt[j] && !((nonu >> j) & 1u) && ft[j] != 0u && (uint64_t)ft[j] < term;
        GF_BAIL(lower && !(cbs[j] & MB_RESP) && (flags & GR_F_CHECK_QUORUM));
        if (lower) {
          fdrop += cnt[j];
        } else if (cnt[j]) {
          L = (uint32_t)j;
          c = cnt[j];
          gl = gin[j];
          go = gout[j];
          cbL = cbs[j];
          nsrc++;
        }
      }
      const uint32_t cc = c < (uint32_t)MK ? c : (uint32_t)MK;
      const bool spec = hf && L == hL;  // the hinted mailbox is the one that sent
      if (c) fmt = ft[L];
      uint64_t fir[MK];
      uint32_t fcr[MK];
#pragma unroll
      for (int k = 0; k < MK; ++k) {  // one batch (keep_value)
        const bool ld = (uint32_t)k < cc && !spec;
        const Mailbox mb = min_at(ld ? gl : 0u);
        fir[k] = ntld(mb.u64(ld ? (uint32_t)k : 0u, MF_LOG_INDEX));
        fcr[k] = ntld(mb.t32(ld ? (uint32_t)k : 0u, MT_CDELTA));
      }
#pragma unroll
      for (int k = 0; k < MK; ++k) {
        const bool ld = (uint32_t)k < cc && !spec;
        const uint64_t a = keep_value(fir[k]);
        const uint32_t b = keep_value(fcr[k]);
        fidx[k] = ld ? a : fidx[k];
        fcd[k] = ld ? b : fcd[k];
      }
      if (mb_shared(cbL)) {  // a shared Replicate pair (MB_SHARED): message 0's fields
        fidx[1] = fidx[0];
        fcd[1] = fcd[0];
      }
      // electionTick = 0 and leaderID = remote_id(L) are usually already so
      // (F_ETZ, F_LSLOT): then neither is loaded nor rewritten
      if (c && ((flags & F_LSLOT) >> F_LSLOT_SHIFT) != L + 1) rid = ntld(s64(Rw::RID + L));
    }
    // ---- checks: anything outside the steady state goes to the general lane
    bool any_input = np != 0;
#pragma unroll
    for (int j = 0; j < S; ++j) any_input = any_input || cnt[j] != 0;
    had_input = any_input;
    GF_BAIL(lw & LW_OTHER);
    if (nq) {
      // QuiescedTick x nq alone (raft.go:431-433: electionTick++ in every
      // state), the bulk of a quiesced population; combined with other
      // inputs it goes to the general lane
      GF_BAIL(any_input);
      if (!ok) return false;
      etick += nq;
      ntst(s64(SR_ETICK), (uint64_t)(etick));
      if (flags & F_ETZ) ntst(s64(SR_HDR), hdr & ~((uint64_t)F_ETZ << H_FLAGS_SHIFT));
#pragma unroll
      for (int j = 0; j < S; ++j)
        if (gout[j] != NOPOS) ntst(mout_at(gout[j]).cnt(), (uint8_t)(0));
      ntst(kp.ln.u8(LR_RFLAGS)[i], (uint8_t)(0));
      GR_COVER(FAST_QUIESCED);
      return true;  // *ls stays zero
    }
    GF_BAIL(!leader && state != GR_FOLLOWER);
    GF_BAIL(np && !leader);
    GF_BAIL(!kLeaderPath && leader && any_input);
    GF_BAIL(!kFollowerPath && !leader && any_input);
    GF_BAIL(any_input && !gelo);  // the window test needs firstIndex-1
    // a non-leader whose remote rows are stale (sync bits) and whose lastIndex
    // may move: the general lane writes the rows out first (Lane::store)
    GF_BAIL(kSync && !(kLeaderPath && leader) && any_input && (hdr & H_SYNC_MASK));
    committed0 = committed;
    hi0 = hi;
    if (kLeaderPath && leader) {
      GF_BAIL(flags & F_LTT);  // leader transfer in progress
#ifdef GR_BAIL_TRACE
      if (ok && nonu) {  // diagnostics: the first message type and flags of each non-uniform mailbox
#pragma unroll
        for (int j = 0; j < S; ++j)
          if ((nonu >> j) & 1u) gr_bail_trace(100000 + 1000 * (int)min_at(gin[j]).type(0) + min_at(gin[j]).flags(0));
      }
#endif
      // a non-uniform mailbox (an old leader's Replicates after an election) is
      // dropped whole when every message in it has a lower term (with checkQuorum,
      // which may ask for a NoOP reply, the check below hands it over)
      uint32_t ndrop = 0;
      if (nonu) {
#pragma unroll
        for (int j = 0; j < S; ++j) {
          if ((nonu >> j) & 1u) {
            GF_BAIL(cnt[j] > (uint32_t)MK || (cbs[j] & MB_COLD_LOST));
            bool low = true;
#pragma unroll
            for (int k = 0; k < MK; ++k) {  // (a slot past the count reads stale words, unused)
              // an MT_WIDE record (a term past 32 bits, gr_host.h encode_msg) has no term word
              const Mailbox mb = min_at(gin[j]);
              const uint32_t ty = ntld(mb.type(k)), tm = ntld(mb.t32(k, MT_TERM));
              low = low && ((uint32_t)k >= cnt[j] || (ty != MT_WIDE && tm != 0u && (uint64_t)tm < term));
            }
            GF_BAIL(!low);
            ndrop |= 1u << j;
          }
        }
      }
      // a uniform mailbox at a lower term is dropped whole (onMessageTermNotMatched,
      // raft.go:1014-1044), unless its messages are Replicates and checkQuorum asks
      // for a NoOP reply; the others must be uniform accepts (ReplicateResp, flags 0)
      // at the current term
      uint32_t drop = 0;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const bool lower = ((ndrop >> j) & 1u) || (cnt[j] && !((nonu >> j) & 1u) && lmt[j] != 0u && (uint64_t)lmt[j] < term);
        GF_BAIL(lower && !(cbs[j] & MB_RESP) && (flags & GR_F_CHECK_QUORUM));
        drop |= lower ? 1u << j : 0u;
        GF_BAIL(!lower && cnt[j] && (cnt[j] > (uint32_t)MK || !(cbs[j] & MB_RESP) || (uint64_t)lmt[j] != term));
      }
      // messages in node.handleReceivedMessages order: slot, then arrival
#pragma unroll
      for (int j = 0; j < S; ++j) {
        if ((drop >> j) & 1u) {
          nmi += cnt[j];
          continue;
        }
#pragma unroll
        for (int k = 0; k < MK; ++k) {
          if ((uint32_t)k < cnt[j]) {
            nmi++;
            if (rkind(j) != GR_SLOT_EMPTY) replicate_resp(j, lidx[j][k]);
          }
        }
      }
      if (np) propose(np);
    } else if (kFollowerPath) {
      // uniform compact Replicates (LogTerm = Term, at most one entry at Term,
      // narrow Commit) from one remote at the current term
      // the source's mailbox may hold full records (a leader's catch-up of several
      // entries, or a LogTerm below its term: emit_replicate, Lane::emit); any
      // other mailbox with messages must be uniform
      const bool fullL = c && ((nonu >> L) & 1u);
      // a full-record mailbox whose cold fields were not delivered (MB_COLD_LOST,
      // gr_space_side_pack) holds a previous pass's words there: CAPACITY in the
      // general lane, as the leader path above and Lane::run do
      GF_BAIL(nsrc > 1 || c > (uint32_t)MK || (nonu & ~(fullL ? 1u << L : 0u)) ||
              (fullL && (cbL & MB_COLD_LOST)) || (c && !fullL && ((cbL & MB_RESP) || (uint64_t)fmt != term)));
      uint32_t ftag[MK], fterm[MK], fn[MK], flt[MK], frt[MK];
      uint64_t fcw[MK];
#pragma unroll
      for (int k = 0; k < MK; ++k) {
        ftag[k] = 0; fterm[k] = 0; fn[k] = 0; flt[k] = 0; frt[k] = 0; fcw[k] = 0;
        if (fullL && (uint32_t)k < c) {  // read_msg's fields (gr_lane.h), one round
          const Mailbox mb = min_at(gl);
          ftag[k] = ntld(mb.tag(k));
          fterm[k] = ntld(mb.t32(k, MT_TERM));
          fn[k] = ntld(mb.n(k));
          flt[k] = ntld(mb.t32(k, MT_LOG_TERM));
          frt[k] = ntld(mb.t32(k, MT_RT0));
          fcw[k] = ntld(mb.u64(k, MF_COMMIT));
        }
      }
      nmi += fdrop;
      uint32_t oc = 0;
#pragma unroll
      for (int k = 0; k < MK; ++k) {
        if ((uint32_t)k < c) {
          nmi++;
          if (fullL) {
            const uint32_t fl = ftag[k] >> 8, runs = (fl >> MFL_RUNS_SHIFT) & 3u;
            // Replicates at the current term with at most one term run; a reject,
            // another type or two runs are the general lane's
            GF_BAIL((ftag[k] & 0xFFu) != GR_REPLICATE || (fl & MFL_REJECT) || runs > 1 || (uint64_t)fterm[k] != term);
            const bool cpt = fl & MFL_COMPACT;
            const uint32_t n = cpt ? ((fl & MFL_N1) ? 1u : 0u) : fn[k];
            GF_BAIL(!cpt && (n ? runs != 1 : runs != 0));
            const uint64_t lt = cpt ? term : (uint64_t)flt[k];
            const uint64_t rt = cpt ? term : (uint64_t)frt[k];
            const uint64_t cm = (!cpt && (fl & MFL_WIDE_COMMIT)) ? fcw[k] : commit_of(fcd[k], fidx[k]);
            replicate(fidx[k], lt, cm, n, n ? rt : 0, go, &oc);
          } else {
            const uint32_t n1 = (cbL >> (MB_N1_SHIFT + k)) & 1u;
            replicate(fidx[k], term, commit_of(fcd[k], fidx[k]), n1, term, go, &oc);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < S; ++j) {
        outc[j] = ((uint32_t)j == L) ? oc : 0u;
      }
    }
    if (!ok) return false;
    // ---- stores (nothing above this line has written state)
    if (committed != committed0) ntst(s64(SR_COMMITTED), (uint64_t)(committed));
    if (hi != hi0) ntst(s64(SR_LAST_INDEX), (uint64_t)(hi));
    uint64_t nh = hdr;  // the header word, rewritten once if anything in it changed
    if (pushed) {
      // right-aligned window: the old newest run moves one row down, the new one
      // takes the last row; it starts above the old newest run, so H_GE_LO holds
      if (nruns > 1) {
        ntst(s64(SR_RUN_START + GR_K - 2), rsn0);
        ntst(s64(SR_RUN_TERM + GR_K - 2), rtn0);
      }
      ntst(s64(SR_RUN_START + GR_K - 1), (uint64_t)(rsn));
      ntst(s64(SR_RUN_TERM + GR_K - 1), (uint64_t)(rtn));
      nh = (nh & ~(7ull << H_NRUNS_SHIFT)) | ((uint64_t)nruns << H_NRUNS_SHIFT) | (1ull << H_GE_LO_BIT);
    }
    if (kLeaderPath && leader) {
      uint64_t rb = h_rb(nh);
      // sync bits: a row in sync with the final lastIndex is not stored (its bit
      // says so); a row that leaves sync, or changed, is
      uint64_t sbits = 0;
      bool all_nx = true, own_ms = false, all_mp = true;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const bool me = (uint32_t)j == self;
        const bool nx_now = kSync && next[j] == hi + 1;
        const bool ms_now = kSync && me && match[j] == hi;
        const bool mp_now = kSync && !me && hi >= 2 && match[j] == hi - 2;
        const bool dj = (mdirty >> j) & 1u;
        const bool m_stale = kSync && (me ? h_ms(hdr) : h_mp(hdr, (uint32_t)j));
        if ((dj || m_stale) && !(me ? ms_now : mp_now)) ntst(s64(Rw::MATCH + j), (uint64_t)(match[j]));
        if ((dj || (kSync && h_nx(hdr, (uint32_t)j))) && !nx_now) ntst(s64(Rw::NEXT + j), (uint64_t)(next[j]));
        sbits |= (nx_now ? 1ull : 0ull) << (H_NX_SHIFT + j);
        sbits |= (ms_now ? 1ull : 0ull) << H_MS_BIT;
        sbits |= (mp_now ? 1ull : 0ull) << (H_MP_SHIFT + j);
        own_ms = own_ms || ms_now;
        if (rkind(j) != GR_SLOT_EMPTY && !nx_now) all_nx = false;
        if (rkind(j) != GR_SLOT_EMPTY && !me && !mp_now) all_mp = false;
      }
      // WH_SYNC (the wave hint): every member's NEXT and MATCH row is stale
      synced = kSync && own_ms && all_nx && all_mp;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        if ((sdirty >> j) & 1u) {
          rb = rb_with(rb, j, 0, 2, rst(j));
          rb = rb_with(rb, j, 2, 1, ract(j));
        }
      }
      nh = (nh & ((1ull << H_REM_SHIFT) - 1)) | (rb << H_REM_SHIFT);
      if (kSync) nh = (nh & ~H_SYNC_MASK) | sbits;
#pragma unroll
      for (int j = 0; j < S; ++j)
        if ((snapz >> j) & 1u) ntst(s64(Rw::SNAP + j), (uint64_t)(0));
    } else if (c) {
      uint32_t nf = flags;
      if (!(flags & F_ETZ)) {
        ntst(s64(SR_ETICK), (uint64_t)(0));  // electionTick = 0 (raft.go:1360)
        nf |= F_ETZ;
      }
      if (((flags & F_LSLOT) >> F_LSLOT_SHIFT) != L + 1) {
        ntst(s64(SR_LEADER_ID), (uint64_t)(rid));  // setLeaderID(m.From)
        nf = (nf & ~F_LSLOT) | ((L + 1) << F_LSLOT_SHIFT);
      }
      nh = (nh & ~(0xFFull << H_FLAGS_SHIFT)) | ((uint64_t)nf << H_FLAGS_SHIFT);
    }
    if (kRuns) {  // run bits (gr_layout.h) after the pass
      uint64_t rbits = 0;
      if (nruns)
        rbits = (rtn == term ? 1ull << H_RTT_BIT : 0ull) |
                ((rknown ? rsn <= committed : true) ? 1ull << H_RLC_BIT : 0ull);  // unknown: rsn <= cload
      nh = (nh & ~H_RUN_MASK) | rbits;
      runs_out = rbits == H_RUN_MASK;
    }
    lslot_out = (h_flags(nh) & F_LSLOT) >> F_LSLOT_SHIFT;
    if (nh != hdr) ntst(s64(SR_HDR), nh);
#pragma unroll
    for (int j = 0; j < S; ++j)
      if (gout[j] != NOPOS) finish_out(j, kLeaderPath && leader);
    uint8_t rf = 0;
    if (prop_result) {  // propose_first = last_index - n + 1 (gr_layout.h)
      rf |= RF_PROPOSE;
      kp.ln.u8(LR_PROP_RESULT)[i] = (uint8_t)prop_result;
    }
    if (append_from) {
      rf |= RF_APPEND;
      kp.ln.u64(LR_APPEND_FROM)[i] = append_from;
    }
    ntst(kp.ln.u8(LR_RFLAGS)[i], (uint8_t)(rf));
    const bool adv = committed > committed0;
    ls->leader_commit = adv && leader;
    ls->follower_commit = adv && !leader;
    ls->escalated = 0;
    ls->msgs_in = nmi;
    ls->msgs_out = nmo;
    ls->leader_in = leader ? nmi : 0;
    ls->leader_out = leader ? nmo : 0;
    ls->entries = nent;
    if (leader) GR_COVER(FAST_LEADER);
    else GR_COVER(FAST_FOLLOWER);
    return true;
  }
  // The lane's role for the next pass's wave hint (WH_*): what it is after this
  // pass when it finished here, what it was when it handed over.
  GF_HD uint32_t role_hint() const {
    if (!had_input) return 0;  // quiesced or idle: nothing to speculate on
    const uint32_t rh = runs_out ? WH_RUNS : 0u;
    if (state == GR_LEADER)
      return WH_LEADER | (self < 8u ? self << WH_SLOT_SHIFT : 0u) | (synced && self < 8u ? WH_SYNC : 0u) | rh;
    if (state != GR_FOLLOWER || !lslot_out) return 0;
    return WH_FOLLOWER | ((lslot_out - 1) << WH_SLOT_SHIFT) | rh;
  }

  // handleReplicateMessage (raft.go:953-976) for an append at the log's end.
  GF_HD void replicate(uint64_t li, uint64_t lterm, uint64_t mcommit, uint32_t n, uint64_t rt0, uint32_t go,
                       uint32_t* oc) {
    nent += n;
    if (li < committed) {
      emit_resp(go, oc, committed, false, 0);
      return;
    }
    if (term_of(li) != lterm) {
      emit_resp(go, oc, li, true, hi);
      return;
    }
    uint64_t ci = 0;
    if (n) {  // getConflictIndex over the newest run (logentry.go:305-312)
      const uint64_t a = li + 1, b = li + n;  // a >= rsn >= firstIndex-1 below (H_GE_LO)
      if (a <= hi) {
        GF_BAIL(nruns == 0 || below_newest(a));
        if (rtn != rt0) ci = a;
      }
      if (ci == 0 && b > hi && rt0 != 0) ci = a > hi + 1 ? a : hi + 1;
    }
    if (ci) {
      GF_BAIL(ci <= committed || ci != hi + 1);  // panic / truncation: general lane
      GF_BAIL(nruns && rknown && rsn > hi);      // a run beyond lastIndex would be truncated
      const uint64_t tprev = (ci - 1 == li) ? lterm : rt0;
      GF_BAIL(tprev > rt0);  // checkEntriesToAppend
      win_push(ci, rt0);
      hi = li + n;
      append_from = append_from ? (append_from < ci ? append_from : ci) : ci;
    }
    const uint64_t last = li + n;
    const uint64_t cm = last < mcommit ? last : mcommit;
    if (cm > committed) {  // commitTo (logentry.go:314-323)
      GF_BAIL(cm > hi);
      committed = cm;
    }
    emit_resp(go, oc, last, false, 0);
  }
};

// The lean lane for lane i (fast_step in gr_steady.h tries the closed-form
// steady lanes first); false = hand the lane to the general kernel.
// *state = the role the lane entered the pass with; *hint_out = its role hint (WH_*).
// take (FastLane::step): a lane whose role is not `take` is left alone, *skipped = true.
template <int S, int R = FL_ANY, int RM = RM_ANY>
GF_HD bool lean_step(const StepParams& kp, uint32_t i, uint32_t p, LaneStats* ls, uint32_t* state = nullptr,
                     uint32_t hint = 0, uint32_t* hint_out = nullptr, int take = FL_ANY,
                     bool* skipped = nullptr) {
  FastLane<S, R, RM> L(kp, i, p, kp.max_entry_size);
  const bool done = L.step(ls, hint, take);
  if (state) *state = L.state;
  if (hint_out) *hint_out = L.role_hint();
  if (skipped) *skipped = L.skipped;
  return done;
}

}  // namespace gr
