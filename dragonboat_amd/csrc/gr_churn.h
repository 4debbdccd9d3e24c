// gr_churn.h — the churn lane: the follower side of a leader change, between
// the lean lanes (gr_fast.h, gr_steady.h) and the general lane (gr_lane.h).
//
// BASELINE config 5 (leader churn) hands the general kernel lanes whose mail
// comes from a new leader: an old leader stepping down on a higher-term
// Replicate, a follower adopting the new term, and the truncating merges and
// below-the-newest-run lookups that follow (bail trace). The
// general lane steps them correctly, but it is built for every handler: its
// register file (256 VGPRs + AGPRs, one wave per SIMD) and its first load round
// (every field group) are what a churn lane pays.
//
// ChurnLane<S> is the general lane's follower path, and only that, composed
// from the same handlers (Lane<S>: term_of over the whole window,
// handle_replicate with getConflictIndex/tryAppend/merge, emit, store), driven
// by its own loop so that nothing else is reachable. Per message, in
// node.handleReceivedMessages order (slot, then arrival):
//   - a higher term (onMessageTermNotMatched raft.go:1014-1044): becomeFollower /
//     becomeObserver (:660-674) with reset (:704-731), the remotes rewritten from
//     lastIndex without loading their rows;
//   - a lower term: dropped, or a NoOP back for a leader message with checkQuorum;
//   - the current term, not leading: Replicate (raft.go:1359-1363 ->
//     handleReplicateMessage :953-976) or Heartbeat (:1365-1369, 923-931).
// Then ProposeEntries of a non-leader (forwarded, handleFollowerPropose
// :1346-1357) and QuiescedTick. Anything else -- a leader's own traffic, a
// candidate, a vote, ticks, ReadIndex, an escalation -- stores nothing and
// returns false: the general lane then steps the lane from its untouched state,
// as it does for the lean lane's hand-overs. So a churn lane's result is the
// general lane's result by construction, with its code and loads cut to the
// follower path (the oracle checks it after every pass: tests/test_hostlane_sim.py
// on the host build, tests/test_device_schedule.py config 5 on the device).
#pragma once
#include "gr_cover.h"
#include "gr_lane.h"

namespace gr {

template <int S>
struct ChurnLane : Lane<S> {
  using L = Lane<S>;
  using L::kp;
  using L::i;
  GR_HD ChurnLane(const StepParams& k, uint32_t lane, uint32_t peer) : L(k, lane, peer) {}

  // raft.reset (raft.go:704-731) for a step-down or term adoption: Lane::reset
  // without loading the remote rows it overwrites (every member slot's match
  // and next follow from lastIndex, snapshotIndex is 0), the FIFO cleared in the
  // header (no entry is live, so no row is written: Lane::store)
  GR_HD int reset(uint64_t t) {
    if (L::rand_used || !kp.has_locals) return GR_ESC_RANDOM;
    L::need(G_CORE | G_TICKS);
    if (L::etimeout == 0) return GR_ESC_PANIC;
    L::rand_used = true;
    const uint64_t rand_value = kp.ln.u64(LR_RAND)[i];
    if (L::term != t) {
      L::term = t;
      L::dirty |= D_TERM | D_VOTE;
    }
    L::leader_id = 0;
    L::loaded |= G_LID;
    L::etick = 0;
    L::loaded |= G_ETICK;
    L::htick = 0;
    L::retimeout = L::etimeout + rand_value % L::etimeout;  // raft.go:435-438
    L::ric = 0;
    L::rifrom = 0;
    L::riack = 0;
    L::loaded |= G_RI;
    L::flags &= ~(uint32_t)GR_F_PENDING_CONFIG_CHANGE;
    L::ltt = 0;  // abortLeaderTransfer: the row is written only if F_LTT said it was set
    L::loaded |= G_LTT;
    L::rb = h_rb(L::hdr0) & ((1ull << (5 * S)) - 1);
    bool empty = false;
#pragma unroll
    for (int j = 0; j < S; ++j) empty = empty || L::rkind((uint32_t)j) == GR_SLOT_EMPTY;
    if (empty) L::need(G_REM);  // an empty slot keeps its rows (as loaded, sync bits resolved)
#pragma unroll
    for (int j = 0; j < S; ++j) {  // resetRemotes/resetObservers :733-753
      if (L::rkind((uint32_t)j) != GR_SLOT_EMPTY) {
        L::next[j] = L::hi + 1;
        L::match[j] = (uint32_t)j == L::self ? L::hi : 0;
        L::set_rstate((uint32_t)j, GR_RETRY);
        L::set_ractive((uint32_t)j, 0);
        L::snapz |= 1u << j;
      }
    }
    L::loaded |= G_REM;
    L::dirty |= D_LEADER | D_ETICK | D_HTICK | D_RETIMEOUT | D_RI | D_FLAGS | D_REM |
                ((L::hdr0 >> H_FLAGS_SHIFT) & F_LTT ? D_LTT : 0u);
    return 0;
  }

  GR_HD int message(const InMsg& m, uint32_t from) {
    const uint32_t t = m.type;
    if (m.term != 0 && m.term != L::term) {  // onMessageTermNotMatched
      if (m.term > L::term) {
        if (t == GR_REQUEST_VOTE) return GR_ESC_UNSUPPORTED;
        const uint64_t lid = is_leader_message(t) ? L::remote_id(from) : 0;
        if (L::state != GR_OBSERVER) {
          L::state = GR_FOLLOWER;
          L::dirty |= D_STATE;
        }
        GR_TRY(reset(m.term));
        L::leader_id = lid;
        GR_COVER(CHURN_ADOPT);
      } else {
        if (is_leader_message(t) && (L::flags & GR_F_CHECK_QUORUM)) {
          OutMsg o;
          o.type = GR_NOOP;
          return L::emit(from, o);
        }
        return 0;  // dropped
      }
    }
    if (L::state != GR_FOLLOWER && L::state != GR_OBSERVER) return GR_ESC_UNSUPPORTED;
    if (t == GR_REPLICATE) {  // raft.go:1359-1363
      L::zero_etick();
      L::set_leader_from(from);
      return L::handle_replicate(m, from);
    }
    if (t == GR_HEARTBEAT) {  // raft.go:1365-1369, 923-931
      L::zero_etick();
      L::set_leader_from(from);
      if (m.commit > L::committed) {
        if (m.commit > L::hi) return GR_ESC_PANIC;
        L::committed = m.commit;
        L::dirty |= D_COMMITTED;
      }
      OutMsg o;
      o.type = GR_HEARTBEAT_RESP;
      o.hint = m.hint;
      o.hint_high = m.hint_high;
      return L::emit(from, o);
    }
    return GR_ESC_UNSUPPORTED;
  }

  // true: the lane's pass is done (state, mailboxes and results stored);
  // false: nothing stored, the general lane steps it
  GR_HD bool step(LaneStats* ls) {
    L::preload();
    L::begin();
    L::need(G_CORE | G_WIN | G_ETICK | G_LID);
    if (L::state == GR_CANDIDATE) return false;
    int e = 0;
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)S && !e; ++j) {
      const uint32_t g = L::in_gpos(j);
      if (g == NOPOS) continue;
      const Mailbox mb = kp.in.at(g);
      const uint32_t cb = GR_LANE_PRELOAD ? L::sel(L::pcb_, j) : (uint32_t)mb.cnt(), c = mb_n(cb);
      if (c > kp.in.depth) e = GR_ESC_CAPACITY;
      if (c && !(cb & MB_UNIFORM) && (cb & MB_COLD_LOST)) e = GR_ESC_CAPACITY;
#pragma unroll 1
      for (uint32_t k = 0; k < c && !e; ++k) {
        InMsg m;
        L::read_msg(mb, cb, k, m);
        if (m.type == MT_WIDE) {
          e = GR_ESC_WIDE_TERM;
          break;
        }
        // a leader's own traffic at its term is the lean and general lanes'
        if (L::state == GR_LEADER && (m.term == 0 || m.term == L::term)) {
          e = GR_ESC_UNSUPPORTED;
          break;
        }
        e = message(m, j);
        L::msgs_in++;
      }
    }
    if (!e && kp.has_locals) {
      const uint32_t lf = L::plf_, nt = L::pnt_, nq = L::pnq_, np = L::pnp_;
      if ((lf & LF_READ_INDEX) || nt) e = GR_ESC_UNSUPPORTED;  // the tick and general lanes'
      if (!e && nq) {  // quiescedTick x nq (raft.go:431-433)
        L::need(G_ETICK);
        L::etick += nq;
        L::dirty |= D_ETICK;
      }
      // a proposal to a lane that no longer leads: handleFollowerPropose /
      // handleObserverPropose (raft.go:1346-1357, 1322), Lane::propose's forward
      if (!e && np) {
        if (L::state == GR_LEADER) {
          e = GR_ESC_UNSUPPORTED;
        } else {
          const bool cc = (lf & LF_PROPOSE_CC) != 0;
          OutMsg o;
          o.type = GR_PROPOSE;
          o.n = np;  // one run of n entries at term 0 (Lane::propose)
          o.flags = (uint8_t)((1u << MFL_RUNS_SHIFT) | (cc ? MFL_REJECT : 0u));
          bool dropped;
          e = L::forward_to_leader(o, &dropped);
          if (dropped) GR_COVER(PROP_DROP_NO_LEADER);
          else GR_COVER(PROP_FORWARD);
          L::prop_result = dropped ? GR_PROP_DROPPED : GR_PROP_FORWARDED;
        }
      }
    }
    if (e) return false;
    GR_COVER(CHURN_FOLLOWER);
    L::store();
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)S; ++j) {  // every routed mailbox is rewritten each pass
      const uint32_t g = L::out_gpos(j);
      if (g == NOPOS) continue;
      const uint32_t c = (L::outcnt >> (3 * j)) & 7u, u = (uint32_t)(L::outu >> (5 * j)) & 31u;
      kp.out.at(g).cnt() = (uint8_t)(c && !(u & 1u) ? c | MB_UNIFORM | ((u & 2u) ? (uint32_t)MB_RESP : 0u) |
                                                         ((u >> 2) << MB_N1_SHIFT)
                                                   : c);
    }
    uint8_t rf = 0;
    if (L::prop_result) {
      rf |= RF_PROPOSE;
      kp.ln.u8(LR_PROP_RESULT)[i] = (uint8_t)L::prop_result;
    }
    if (L::append_from) {
      rf |= RF_APPEND;
      kp.ln.u64(LR_APPEND_FROM)[i] = L::append_from;
    }
    if (L::dirty & (D_TERM | D_VOTE)) rf |= RF_HARDSTATE;
    kp.ln.u8(LR_RFLAGS)[i] = rf;
    const bool adv = (L::dirty & D_COMMITTED) && L::committed > L::committed0;
    ls->leader_commit = 0;
    ls->follower_commit = adv;
    ls->escalated = 0;
    ls->msgs_in = L::msgs_in;
    ls->msgs_out = L::msgs_out;
    ls->leader_in = 0;
    ls->leader_out = 0;
    ls->entries = L::entries_in;
    return true;
  }
};

template <int S>
GR_HD bool churn_step(const StepParams& kp, uint32_t i, uint32_t p, LaneStats* ls) {
  ChurnLane<S> C(kp, i, p);
  return C.step(ls);
}

}  // namespace gr
