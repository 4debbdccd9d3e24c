// gr_steady.h — closed-form steady-state lanes of the lean kernel.
//
// Measured (profiles/r03_a, SQ counters): the lean kernel instances are bound
// by vector-instruction issue, not by HBM. A leader wave executed ~1,100 VALU
// and ~1,000 SALU instructions, a follower wave ~650 and ~530: at 4 cycles per
// wave64 VALU instruction that is 28 of the leader instance's 48 us and 33 of
// the follower instance's 49 us. Most of them are the general control flow of
// FastLane (gr_fast.h), which handles any remote state, observers, pauses,
// rejects and window pushes, and inlines a broadcast per message.
//
// In the steady state almost none of that can happen, and the whole pass has
// a closed form. A wave whose hint says it was steady at the end of the last
// pass (WH_LEADER | WH_SYNC | WH_RUNS, or WH_FOLLOWER | WH_RUNS) runs one of
// the two lanes below first. Each issues its loads in one round, checks the
// preconditions under which the closed form equals FastLane's result (and so
// the reference's), and stores only if they hold. Otherwise it stores nothing
// and the lane runs FastLane from its untouched state.
//
// SteadyLeader<S = 3>: handleLeaderReplicateResp (raft.go:1205-1227) for
// uniform accepts at the current term from followers in the Replicate state,
// then handleLeaderPropose (raft.go:1125-1146) of at most one entry.
// Preconditions: every slot a voter; the followers Replicate, active, with
// next = lastIndex + 1 (sync bits); match[self] = lastIndex; the newest term
// run at the current term starting at or below committed (run bits); no leader
// transfer; every ack at or below lastIndex. Then per ack, in
// node.handleReceivedMessages order (slot, then arrival):
//   remote.tryUpdate (remote.go:108-118) only raises match (next stays
//   lastIndex + 1, respondedTo is a no-op in Replicate);
//   tryCommit (raft.go:625-641) = the median of the three match values, whose
//   term is the current term whenever it is above committed;
//   a commit broadcasts an empty Replicate {LogIndex = lastIndex, LogTerm =
//   term, Commit} to both followers (makeReplicateMessage, raft.go:474-498:
//   next > lastIndex, so no entries, and progress leaves next unchanged).
// The proposal appends at lastIndex + 1 without a new term run, moves
// match/next of self, and broadcasts one Replicate of one entry
// {LogIndex = old lastIndex, LogTerm = term, Commit}; progress moves every
// follower's next to the new lastIndex + 1, so the sync bits stay exact.
//
// SteadyFollower<S>: handleReplicateMessage (raft.go:953-976) for the uniform
// compact Replicates of the leader slot L at the current term, with
// electionTick already 0 and leaderID already L's node (F_ETZ, F_LSLOT), run
// bits set, no sync bits and no local input. For each Replicate:
//   LogIndex < committed: accept at committed (raft.go:958-961);
//   else LogIndex <= lastIndex, so matchTerm holds (the run bits put every
//   index at or above committed in the newest run, at the current term); an
//   entry at LogIndex + 1 <= lastIndex matches too (getConflictIndex
//   logentry.go:305-312: no conflict), one at lastIndex + 1 appends
//   (tryAppend :281-292, no new run); commitTo(min(last, Commit)); accept.
//   LogIndex > lastIndex is a reject (matchTerm fails): FastLane's.
#pragma once
#include "gr_cover.h"
#include "gr_fast.h"
#include "gr_layout.h"

namespace gr {

// The wave hints that select the steady lanes.
constexpr uint32_t WH_STEADY_LEADER = WH_LEADER | WH_SYNC | WH_RUNS;
__host__ __device__ inline bool steady_leader_hint(uint32_t h) {
  return (h & (WH_ROLE | WH_SYNC | WH_RUNS)) == WH_STEADY_LEADER;
}
__host__ __device__ inline bool steady_follower_hint(uint32_t h) {
  return (h & (WH_ROLE | WH_RUNS)) == (WH_FOLLOWER | WH_RUNS);
}
// A hint for which S has a steady lane (leaders: S = 3 only).
template <int S>
__host__ __device__ inline bool steady_hint(uint32_t h) {
  return (S == 3 && steady_leader_hint(h)) || steady_follower_hint(h);
}

template <int RM>
struct SteadyBase {
  static constexpr bool kOneChunk = RM == RT_LOOPBACK;
  const StepParams& kp;
  const uint32_t i, p;
  GF_HD SteadyBase(const StepParams& k, uint32_t lane, uint32_t peer) : kp(k), i(lane), p(peer) {}
  GF_HD uint64_t& s64(uint32_t row) const { return kp.st.u64(row)[p]; }
  GF_HD Mailbox min_at(uint32_t g) const { return kp.in.template at<kOneChunk>(g); }
  GF_HD Mailbox mout_at(uint32_t g) const { return kp.out.template at<kOneChunk>(g); }
  GF_HD static uint64_t umin(uint64_t a, uint64_t b) { return a < b ? a : b; }
  GF_HD static uint64_t umax(uint64_t a, uint64_t b) { return a < b ? b : a; }
};

template <int S, int RM>
struct SteadyLeader : SteadyBase<RM> {
  using B = SteadyBase<RM>;
  using B::kp;
  using B::i;
  using Rw = Rows<S>;
  static_assert(S == 3, "the closed form is the median of three voters");
  GF_HD SteadyLeader(const StepParams& k, uint32_t lane, uint32_t peer) : B(k, lane, peer) {}

  // true: the pass is done (state, messages, results stored); false: nothing stored.
  GF_HD bool step(LaneStats* ls, uint32_t hint, uint32_t* hint_out) {
    const uint32_t hself = (hint >> WH_SLOT_SHIFT) & 7u;  // wave-uniform
    uint32_t gin[S], gout[S];
    routes_of<S, RM>(kp, i, gin, gout);
    // ---- one load round
    const uint64_t hdr = ntld(B::s64(SR_HDR));
    const uint64_t term = ntld(B::s64(SR_TERM));
    const uint64_t committed0 = ntld(B::s64(SR_COMMITTED));
    const uint64_t hi0 = ntld(B::s64(SR_LAST_INDEX));
    const uint32_t lw = kp.has_locals ? ntld(kp.ln.u32(LR_LWORD)[i]) : 0u;
    uint32_t cb[S], mt[S];
    uint64_t x[S][2], m[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const bool in = gin[j] != NOPOS;
      const Mailbox mb = B::min_at(in ? gin[j] : 0u);
      cb[j] = in ? (uint32_t)ntld(mb.cnt()) : 0u;
      mt[j] = in ? ntld(mb.mterm()) : 0u;
      x[j][0] = in ? ntld(mb.u64(0, MF_LOG_INDEX)) : 0ull;
      m[j] = (uint32_t)j != hself ? hi0 - 2 : hi0;  // H_MP / H_MS (checked below): no MATCH row loaded
    }
    // a second ack: shared mailboxes (MB_SHARED, the steady state) imply it from
    // the first; only an unshared pair loads it, in a second round
#pragma unroll
    for (int j = 0; j < S; ++j) {
      x[j][1] = x[j][0] + 1;
      if (gin[j] != NOPOS && mb_n(cb[j]) >= 2 && !mb_shared(cb[j]))
        x[j][1] = ntld(B::min_at(gin[j]).u64(1, MF_LOG_INDEX));
    }
    // ---- preconditions (see the header comment)
    const uint32_t self = h_self(hdr), flags = h_flags(hdr);
    const uint64_t rb = h_rb(hdr);
    const uint32_t np = lw & 0xFFFFu;
    bool ok = h_state(hdr) == GR_LEADER && self == hself && h_nruns(hdr) >= 1 && h_gelo(hdr) &&
              (hdr & H_RUN_MASK) == H_RUN_MASK && h_ms(hdr) && !(flags & F_LTT) && !wide_term(term, 0, 0, 0) &&
              (lw & ~0xFFFFu) == 0 && np <= 1;
    uint32_t nmi = 0;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      ok = ok && rb_kind(rb, j) == GR_SLOT_VOTER && h_nx(hdr, j);
      const uint32_t c = mb_n(cb[j]);
      nmi += c;
      if ((uint32_t)j != hself) {
        ok = ok && h_mp(hdr, j) && rb_state(rb, j) == GR_REPLICATE_ST && rb_active(rb, j);
        ok = ok && (c == 0 || ((cb[j] & MB_UNIFORM) && (cb[j] & MB_RESP) && c <= 2 && (uint64_t)mt[j] == term));
        ok = ok && (c < 1 || x[j][0] <= hi0) && (c < 2 || x[j][1] <= hi0);
      } else {
        ok = ok && c == 0;
      }
    }
    // ---- the acks, in slot then arrival order: tryUpdate, tryCommit
    uint64_t c = committed0;
    uint64_t bc0 = 0, bc1 = 0;  // the Commit of the first / second commit broadcast
    uint32_t ncb = 0;
#pragma unroll
    for (int j = 0; j < S; ++j) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const bool upd = (uint32_t)j != hself && (uint32_t)k < mb_n(cb[j]) && m[j] < x[j][k];
        m[j] = upd ? x[j][k] : m[j];
        const uint64_t q = B::umax(B::umin(m[0], m[1]), B::umin(B::umax(m[0], m[1]), m[2]));  // sortMatchValues, R = 3
        const bool adv = upd && q > c;
        bc0 = adv && ncb == 0 ? q : bc0;
        bc1 = adv && ncb == 1 ? q : bc1;
        ncb += adv ? 1u : 0u;
        c = adv ? q : c;
      }
    }
    const uint32_t nout = ncb + np;  // messages per follower mailbox
    // the closed form keeps two commit broadcasts (bc0, bc1): a third one (staggered
    // acks, e.g. A acks 10, 11 and B acks 12 over committed 9) is FastLane's
    ok = ok && ncb <= 2 && nout <= kUniformMax && nout <= kp.out.depth;
    uint32_t cd0 = 0, cd1 = 0, cdp = 0;
    ok = ok && (ncb < 1 || commit_delta(bc0, hi0, &cd0)) && (ncb < 2 || commit_delta(bc1, hi0, &cd1)) &&
         (np == 0 || commit_delta(c, hi0, &cdp));
#pragma unroll
    for (int j = 0; j < S; ++j) ok = ok && ((uint32_t)j == hself || nout == 0 || gout[j] != NOPOS);
    if (!ok) return false;
    // ---- stores
    const uint64_t hi = hi0 + np;  // the proposal's entry (no new run: the newest one is at term)
    if (c != committed0) ntst(B::s64(SR_COMMITTED), c);
    if (np) ntst(B::s64(SR_LAST_INDEX), hi);
    // match[self] = lastIndex and every next = lastIndex + 1 again (H_MS, H_NX
    // hold); a follower's match is lastIndex - 2 again when its acks were for the
    // entry two proposals back (H_MP holds, nothing stored), else its row is
    // written and its bit cleared
    uint64_t nh = hdr;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      if ((uint32_t)j == hself || m[j] == hi - 2) continue;
      ntst(B::s64(Rw::MATCH + j), m[j]);
      nh &= ~(1ull << (H_MP_SHIFT + j));
    }
    if (nh != hdr) ntst(B::s64(SR_HDR), nh);
    // one commit broadcast and the proposal: both carry LogIndex = the old
    // lastIndex and Commit = c, a shared mailbox (gr_layout.h MB_SHARED) stores
    // message 0's fields only
    const bool shared = ncb == 1 && np == 1;
    const uint32_t nb = nout | MB_UNIFORM | (shared ? MB_SHARED : 0u) | (np ? 1u << (MB_N1_SHIFT + ncb) : 0u);
#pragma unroll
    for (int j = 0; j < S; ++j) {
      if (gout[j] == NOPOS) continue;
      const Mailbox mb = B::mout_at(gout[j]);
      if ((uint32_t)j == hself || nout == 0) {
        ntst(mb.cnt(), (uint8_t)0);
        continue;
      }
      // every Replicate of this pass has LogIndex = the old lastIndex
      if (ncb > 0) {
        ntst(mb.u64(0, MF_LOG_INDEX), hi0);
        ntst(mb.t32(0, MT_CDELTA), cd0);
      }
      if (ncb > 1) {
        ntst(mb.u64(1, MF_LOG_INDEX), hi0);
        ntst(mb.t32(1, MT_CDELTA), cd1);
      }
      if (np && !shared) {
        ntst(mb.u64(ncb, MF_LOG_INDEX), hi0);
        ntst(mb.t32(ncb, MT_CDELTA), cdp);
      }
      ntst(mb.mterm(), (uint32_t)term);
      ntst(mb.cnt(), (uint8_t)nb);
    }
    if (np) kp.ln.u8(LR_PROP_RESULT)[i] = (uint8_t)GR_PROP_APPENDED;
    ntst(kp.ln.u8(LR_RFLAGS)[i], (uint8_t)(np ? RF_PROPOSE : 0));
    const uint32_t nmo = nout * (S - 1);
    ls->leader_commit = c > committed0;
    ls->follower_commit = 0;
    ls->escalated = 0;
    ls->msgs_in = nmi;
    ls->msgs_out = nmo;
    ls->leader_in = nmi;
    ls->leader_out = nmo;
    ls->entries = 0;
    // FastLane::role_hint: WH_SYNC only while every member row is stale
    *hint_out = (nmi || np) ? ((nh == hdr ? WH_STEADY_LEADER : (WH_LEADER | WH_RUNS)) | (self << WH_SLOT_SHIFT)) : 0u;
    GR_COVER(STEADY_LEADER);
    return true;
  }
};

template <int S, int RM>
struct SteadyFollower : SteadyBase<RM> {
  using B = SteadyBase<RM>;
  using B::kp;
  using B::i;
  GF_HD SteadyFollower(const StepParams& k, uint32_t lane, uint32_t peer) : B(k, lane, peer) {}

  GF_HD bool step(LaneStats* ls, uint32_t hint, uint32_t* hint_out) {
    const uint32_t hL = (hint >> WH_SLOT_SHIFT) & 7u;  // wave-uniform: the leader's slot
    uint32_t gin[S], gout[S];
    routes_of<S, RM>(kp, i, gin, gout);
    // ---- one load round
    const uint64_t hdr = ntld(B::s64(SR_HDR));
    const uint64_t term = ntld(B::s64(SR_TERM));
    const uint64_t committed0 = ntld(B::s64(SR_COMMITTED));
    const uint64_t hi0 = ntld(B::s64(SR_LAST_INDEX));
    const uint32_t lw = kp.has_locals ? ntld(kp.ln.u32(LR_LWORD)[i]) : 0u;
    uint32_t other = 0;  // messages from any slot but hL
    uint32_t gL = NOPOS, oL = NOPOS;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const bool in = gin[j] != NOPOS;
      const uint32_t b = in ? (uint32_t)ntld(B::min_at(gin[j]).cnt()) : 0u;
      other |= (uint32_t)j != hL ? mb_n(b) : 0u;
      gL = (uint32_t)j == hL ? gin[j] : gL;
      oL = (uint32_t)j == hL ? gout[j] : oL;
    }
    const Mailbox mb = B::min_at(gL != NOPOS ? gL : 0u);
    const uint32_t cbL = gL != NOPOS ? (uint32_t)ntld(mb.cnt()) : 0u;
    const uint32_t fmt = gL != NOPOS ? ntld(mb.mterm()) : 0u;
    uint64_t li[2];
    uint32_t cd[2];
    li[0] = gL != NOPOS ? ntld(mb.u64(0, MF_LOG_INDEX)) : 0ull;
    cd[0] = gL != NOPOS ? ntld(mb.t32(0, MT_CDELTA)) : 0u;
    // a shared mailbox (MB_SHARED, the steady state) repeats message 0's fields;
    // only an unshared pair loads the second, in a second round
    li[1] = li[0];
    cd[1] = cd[0];
    if (gL != NOPOS && mb_n(cbL) >= 2 && !mb_shared(cbL)) {
      li[1] = ntld(mb.u64(1, MF_LOG_INDEX));
      cd[1] = ntld(mb.t32(1, MT_CDELTA));
    }
    // ---- preconditions
    const uint32_t flags = h_flags(hdr);
    const uint32_t c = mb_n(cbL);
    // the sync bits exist for S <= 3 only: above that, bits 40-59 are remote
    // slots' rb fields (gr_layout.h), which a follower's voters always set
    bool ok = h_state(hdr) == GR_FOLLOWER && !(has_sync_bits(S) && (hdr & H_SYNC_MASK)) &&
              (hdr & H_RUN_MASK) == H_RUN_MASK &&
              h_nruns(hdr) >= 1 && h_gelo(hdr) && (flags & F_ETZ) && ((flags & F_LSLOT) >> F_LSLOT_SHIFT) == hL + 1 &&
              lw == 0 && other == 0 && !wide_term(term, 0, 0, 0);
    ok = ok && (c == 0 || ((cbL & MB_UNIFORM) && !(cbL & MB_RESP) && c <= 2 && (uint64_t)fmt == term));
    ok = ok && (c == 0 || (oL != NOPOS && c <= kp.out.depth));
    // ---- the Replicates, in arrival order
    uint64_t committed = committed0, hi = hi0, append_from = 0, out[2];
    uint32_t nent = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const bool v = (uint32_t)k < c;
      const uint32_t n1 = v ? (cbL >> (MB_N1_SHIFT + k)) & 1u : 0u;
      nent += n1;
      const bool early = li[k] < committed;  // raft.go:958-961
      ok = ok && (!v || early || li[k] <= hi);  // above lastIndex: matchTerm fails, a reject
      const uint64_t a = li[k] + 1;
      const bool app = v && !early && n1 && a > hi;  // the entry lands at lastIndex + 1
      append_from = app ? (append_from ? B::umin(append_from, a) : a) : append_from;
      hi = app ? a : hi;
      const uint64_t last = li[k] + n1;
      const uint64_t cm = B::umin(last, commit_of(cd[k], li[k]));
      committed = v && !early && cm > committed ? cm : committed;
      out[k] = early ? committed : last;
    }
    if (!ok) return false;
    // ---- stores
    if (committed != committed0) ntst(B::s64(SR_COMMITTED), committed);
    if (hi != hi0) ntst(B::s64(SR_LAST_INDEX), hi);
#pragma unroll
    for (int j = 0; j < S; ++j) {
      if (gout[j] == NOPOS) continue;
      const Mailbox mo = B::mout_at(gout[j]);
      if ((uint32_t)j != hL || c == 0) {
        ntst(mo.cnt(), (uint8_t)0);
        continue;
      }
      // two consecutive accepts (the acks of a commit broadcast and the proposal
      // after it) make a shared mailbox: LogIndex of message 0 only
      const bool shared = c == 2 && out[1] == out[0] + 1;
      ntst(mo.u64(0, MF_LOG_INDEX), out[0]);
      if (c > 1 && !shared) ntst(mo.u64(1, MF_LOG_INDEX), out[1]);
      ntst(mo.mterm(), (uint32_t)term);
      ntst(mo.cnt(), (uint8_t)(c | MB_UNIFORM | MB_RESP | (shared ? MB_SHARED : 0u)));
    }
    if (append_from) kp.ln.u64(LR_APPEND_FROM)[i] = append_from;
    ntst(kp.ln.u8(LR_RFLAGS)[i], (uint8_t)(append_from ? RF_APPEND : 0));
    ls->leader_commit = 0;
    ls->follower_commit = committed > committed0;
    ls->escalated = 0;
    ls->msgs_in = c;
    ls->msgs_out = c;
    ls->leader_in = 0;
    ls->leader_out = 0;
    ls->entries = nent;
    *hint_out = c ? (WH_FOLLOWER | WH_RUNS | (hL << WH_SLOT_SHIFT)) : 0u;  // FastLane::role_hint
    GR_COVER(STEADY_FOLLOWER);
    return true;
  }
};

// What the steady kernel did with a lane of a wave whose hint is not steady
// (gr_kernels.h gr_steady_kernel): finished it, sent it to the tick lists, or
// left it to the role instances.
constexpr int QS_DONE = 0, QS_TICK = 1, QS_OTHER = 2;

// QuiescedTick x nq alone (raft.go:431-433: electionTick++ in every state, one
// item), FastLane's quiesced path (gr_fast.h) in closed form: no message in any
// in-mailbox, no proposal, no tick or ReadIndex. Quiesced populations carry no
// role hint (a wave of quiet groups has no input to speculate on), so their
// lanes would otherwise all go through the role instances.
// stage (a lane with ticks or a ReadIndex, QS_TICK): its TickStage words (the
// header, electionTick, locals word and count bytes, loaded here with the
// wave's quiesced lanes), and its out counts zeroed here (coalesced with theirs;
// the tick lane then writes only the mailboxes it fills).
template <int S, int RM>
GF_HD int quiet_step(const StepParams& kp, uint32_t i, uint32_t p, uint64_t* stage, bool do_stage) {  // lane i, peer p
  constexpr bool kOneChunk = RM == RT_LOOPBACK;
  if (!kp.has_locals) return QS_OTHER;
  const uint32_t lw = ntld(kp.ln.u32(LR_LWORD)[i]);
  const bool tick = (lw & LW_OTHER) != 0;
  if (tick && !do_stage) return QS_TICK;
  const uint32_t np = lw & 0xFFFFu, nq = (lw >> LW_QT_SHIFT) & LW_QT_MAX;
  if (!tick && (!nq || np)) return QS_OTHER;
  uint32_t gin[S], gout[S];
  routes_of<S, RM>(kp, i, gin, gout);
  const uint64_t hdr = ntld(kp.st.u64(SR_HDR)[p]), et = ntld(kp.st.u64(SR_ETICK)[p]);
  uint32_t any = 0;
  uint64_t cw = 0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const uint32_t b = gin[j] != NOPOS ? (uint32_t)ntld(kp.in.template at<kOneChunk>(gin[j]).cnt()) : 0u;
    any |= mb_n(b);
    cw |= (uint64_t)(b & 0xFFu) << (8 * j);
  }
  if (tick) {
    stage[0] = hdr;
    stage[1] = et;
    stage[2] = lw | ((uint64_t)kp.pass_tag << 32);
    stage[3] = cw;
#pragma unroll
    for (int j = 0; j < S; ++j)
      if (gout[j] != NOPOS) ntst(kp.out.template at<kOneChunk>(gout[j]).cnt(), (uint8_t)0);
    return QS_TICK;
  }
  if (any) return QS_OTHER;
  ntst(kp.st.u64(SR_ETICK)[p], (uint64_t)(et + nq));
  if (h_flags(hdr) & F_ETZ) ntst(kp.st.u64(SR_HDR)[p], hdr & ~((uint64_t)F_ETZ << H_FLAGS_SHIFT));
#pragma unroll
  for (int j = 0; j < S; ++j)
    if (gout[j] != NOPOS) ntst(kp.out.template at<kOneChunk>(gout[j]).cnt(), (uint8_t)0);
  ntst(kp.ln.u8(LR_RFLAGS)[i], (uint8_t)0);
  GR_COVER(QUIET_STEP);
  return QS_DONE;
}

// A lane of an unhinted wave with messages or a proposal (quiet_step's
// QS_OTHER): the closed form of the role its own header names, with the slot a
// wave hint would carry read from the header (a leader's own slot; a follower's
// leader slot, F_LSLOT). A wave whose groups' leaders sit on different replicas
// (elections, config 5's leader changes) has no common hint, and without this
// every lane of it ran FastLane. The closed forms check every precondition, the
// slot included, against the lane's state, so a lane that fails them has stored
// nothing (false) and goes on to FastLane.
#ifndef GR_LANE_CLOSED
#define GR_LANE_CLOSED 1  // the steady kernel tries it on unhinted waves (A/B builds: 0)
#endif
template <int S, int RM>
GF_HD bool lane_closed_form(const StepParams& kp, uint32_t i, uint32_t p, LaneStats* ls, uint32_t* role,
                            uint32_t* hint_out) {
  const uint64_t hdr = kp.st.u64(SR_HDR)[p];
  const uint32_t st = h_state(hdr);
  if constexpr (S == 3) {
    if (st == GR_LEADER) {
      *role = GR_LEADER;
      return SteadyLeader<S, RM>(kp, i, p).step(ls, WH_STEADY_LEADER | (h_self(hdr) << WH_SLOT_SHIFT), hint_out);
    }
  }
  const uint32_t sl = (h_flags(hdr) & F_LSLOT) >> F_LSLOT_SHIFT;  // the leader's slot + 1, 0: none known
  if (st != GR_FOLLOWER || sl == 0 || sl > (uint32_t)S) return false;
  *role = GR_FOLLOWER;
  return SteadyFollower<S, RM>(kp, i, p).step(ls, WH_FOLLOWER | WH_RUNS | ((sl - 1) << WH_SLOT_SHIFT), hint_out);
}

// Kernel-side entry (gr_kernels.h, and the host build of the lane): a wave
// hinted steady runs the closed-form lane of its role first; any lane it does
// not finish (nothing stored) runs FastLane; false = hand the lane to the
// general kernel. Arguments as lean_step (gr_fast.h).
template <int S, int R = FL_ANY, int RM = RM_ANY>
GF_HD bool fast_step(const StepParams& kp, uint32_t i, uint32_t p, LaneStats* ls, uint32_t* state = nullptr,
                     uint32_t hint = 0, uint32_t* hint_out = nullptr, int take = FL_ANY,
                     bool* skipped = nullptr) {
  if (take == FL_ANY) {
    uint32_t h = 0;
    bool done = false, lead = false;
    if constexpr (S == 3 && R != FL_FOLLOWER) {
      if (steady_leader_hint(hint)) {
        done = SteadyLeader<S, RM>(kp, i, p).step(ls, hint, &h);
        lead = true;
      }
    }
    if constexpr (R != FL_LEADER) {
      if (!done && steady_follower_hint(hint)) done = SteadyFollower<S, RM>(kp, i, p).step(ls, hint, &h);
    }
    if (done) {
      if (state) *state = lead ? GR_LEADER : GR_FOLLOWER;
      if (hint_out) *hint_out = h;
      if (skipped) *skipped = false;
      return true;
    }
  }
  return lean_step<S, R, RM>(kp, i, p, ls, state, hint, hint_out, take, skipped);
}

}  // namespace gr
