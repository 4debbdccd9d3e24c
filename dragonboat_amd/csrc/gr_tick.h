// gr_tick.h — the lean lane for heartbeat, ReadIndex and tick traffic: the
// north-star's ReadIndex quorum-ack reduction and election/heartbeat tick
// sweep, for lanes the steady-state lane (gr_fast.h) hands over.
//
//   follower: Heartbeats at the current term from one remote (raft.go:1365-1369,
//             handleHeartbeatMessage :923-931: electionTick = 0, leaderID,
//             commitTo(m.Commit), HeartbeatResp echoing the context), then
//             Tick x n without reaching the randomized election timeout
//             (nonLeaderTick :386-401);
//   leader:   HeartbeatResps at the current term from caught-up remotes
//             (handleLeaderHeartbeatResp :1229-1240 + readIndex.confirm,
//             readindex.go:77-116: ack bit, popcount quorum test, prefix
//             release into ReadyToRead), a local ReadIndex (handleLeaderReadIndex
//             :1171-1203: readIndex.addRequest + broadcastHeartbeatMessageWithHint
//             :575-587), then at most one Tick (leaderTick :403-429 with
//             CheckQuorum :1117-1123, 262-271 and the heartbeat broadcast).
// It restates that subset of the general lane (gr_lane.h) with compile-time
// remote slots. Anything else (an election or step-down, a lagging remote, a
// ReadIndex from another node, FIFO or mailbox capacity, other inputs) clears
// `ok`; the lane then stores no state and the general lane steps it. It runs in
// the general kernel, in front of the general lane, on the lanes pass 1 handed
// over, so it costs the steady-state kernel nothing.
#pragma once
#include "gr_cover.h"
#include "gr_layout.h"

namespace gr {

#define GT_HD __host__ __device__ inline __attribute__((always_inline))
#define GT_BAIL(c) (ok = ok ? !(c) && ok : false)

GT_HD uint32_t gt_popc8(uint32_t x) {
  x &= 0xFFu;
  x = x - ((x >> 1) & 0x55u);
  x = (x & 0x33u) + ((x >> 2) & 0x33u);
  return (x + (x >> 4)) & 0x0Fu;
}

template <int S, int RM = RM_ANY>
struct TickLane {
  using Rw = Rows<S>;
  static constexpr int MK = 2;  // messages per mailbox handled here

  const StepParams& kp;
  const uint32_t i, p;
  bool ok = true;
  uint64_t hdr = 0;
  uint32_t state = 0, self = 0, flags = 0, nruns = 0;
  bool gelo = false;
  uint64_t term = 0, committed = 0, committed0 = 0, hi = 0, rsn = 0, rtn = 0, rclo = 0, rchi = 0;
  uint64_t etick = 0, etick0 = 0;
  // leader
  uint64_t match[S];
  uint32_t rst[S], ract[S], rkind[S], sdirty = 0;
  uint64_t htick = 0, htick0 = 0, etimeout = 0, htimeout = 0;
  uint32_t ric = 0, rifrom = 0, riack = 0;
  uint64_t rii[GR_Q], rilo[GR_Q], rihi[GR_Q];
  bool fifo_dirty = false;
  uint32_t rtrc = 0;
  uint64_t rdi[GR_Q], rdl[GR_Q], rdh[GR_Q];
  // emission
  uint32_t gout[S], outc[S];
  uint32_t nmi = 0, nmo = 0;

  uint64_t tclk[3] = {0, 0, 0};  // GR_WAVE_CLOCK marks: round 1 in, round 2 in, stores issued
  const uint64_t* stage;  // the entry's TickStage record, or nullptr
  bool staged = false;    // ... written this pass: the out counts are zero already
  GT_HD TickLane(const StepParams& k, uint32_t lane, uint32_t peer, const uint64_t* stg = nullptr)
      : kp(k), i(lane), p(peer), stage(stg) {}
  GT_HD uint64_t& s64(uint32_t row) const { return kp.st.u64(row)[p]; }
  GT_HD uint8_t& s8(uint32_t row) const { return kp.st.u8(row)[p]; }

  GT_HD void emit(int j, uint8_t type, uint64_t commit, uint64_t hint, uint64_t hint_high) {
    GT_BAIL(gout[j] == NOPOS || outc[j] >= kp.out.depth || wide_term(term, 0, 0, 0));
    if (!ok) return;
    const Mailbox mb = kp.out.at(gout[j]);
    const uint32_t c = outc[j];
    mb.type(c) = type;
    mb.flags(c) = 0;
    mb.t32(c, MT_TERM) = (uint32_t)term;
    if (type == GR_HEARTBEAT) mb.u64(c, MF_COMMIT) = commit;
    mb.u64(c, MF_HINT) = hint;
    mb.u64(c, MF_HINT_HIGH) = hint_high;
    outc[j] = c + 1;
    nmo++;
  }
  GT_HD int quorum() const {
    int nv = 0;
#pragma unroll
    for (int j = 0; j < S; ++j) nv += rkind[j] == GR_SLOT_VOTER;
    return nv / 2 + 1;
  }
  GT_HD void add_ready(uint64_t index, uint64_t lo, uint64_t hi_) {  // raft.go:1163-1169
    GT_BAIL(rtrc >= (uint32_t)GR_Q);
    if (!ok) return;
#pragma unroll
    for (int q = 0; q < GR_Q; ++q) {
      const bool hit = (uint32_t)q == rtrc;
      rdi[q] = hit ? index : rdi[q];
      rdl[q] = hit ? lo : rdl[q];
      rdh[q] = hit ? hi_ : rdh[q];
    }
    rtrc++;
  }
  // broadcastHeartbeatMessageWithHint (raft.go:575-587)
  GT_HD void broadcast_heartbeat(uint64_t clo, uint64_t chi) {
#pragma unroll
    for (int j = 0; j < S; ++j)
      if (rkind[j] == GR_SLOT_VOTER && (uint32_t)j != self)
        emit(j, GR_HEARTBEAT, match[j] < committed ? match[j] : committed, clo, chi);
    if (clo == 0 && chi == 0) {
#pragma unroll
      for (int j = 0; j < S; ++j)
        if (rkind[j] == GR_SLOT_OBSERVER) emit(j, GR_HEARTBEAT, match[j] < committed ? match[j] : committed, 0, 0);
    }
  }
  // readIndex.confirm + handleReadIndexLeaderConfirmation (readindex.go:77-116, raft.go:1264-1284)
  GT_HD void ri_confirm(uint64_t clo, uint64_t chi, uint32_t from) {
    int pos = -1;
#pragma unroll
    for (int q = 0; q < GR_Q; ++q)
      pos = (pos < 0 && (uint32_t)q < ric && rilo[q] == clo && rihi[q] == chi) ? q : pos;
    if (pos < 0) return;
    riack |= (1u << from) << (8 * pos);
    fifo_dirty = true;
    const uint32_t ack = (riack >> (8 * pos)) & 0xFFu;
    if ((int)gt_popc8(ack) + 1 < quorum()) return;
    uint64_t sidx = 0;
#pragma unroll
    for (int q = 0; q < GR_Q; ++q) sidx = (q == pos) ? rii[q] : sidx;
#pragma unroll
    for (int q = 0; q < GR_Q; ++q) {
      if (q <= pos) {
        GT_BAIL(rii[q] > sidx);  // panic in the reference
        const uint32_t f = (rifrom >> (8 * q)) & 0xFFu;
        GT_BAIL(f != GR_SLOT_NONE && f != self);  // ReadIndexResp to another node: general lane
        add_ready(sidx, rilo[q], rihi[q]);
      }
    }
    const uint32_t drop = (uint32_t)pos + 1;
#pragma unroll
    for (int q = 0; q < GR_Q; ++q) {  // queue = queue[done:]
      uint64_t a = 0, b = 0, c = 0;
#pragma unroll
      for (int d = 1; d + q < GR_Q; ++d) {
        const bool hit = (uint32_t)d == drop;
        a = hit ? rii[q + d] : a;
        b = hit ? rilo[q + d] : b;
        c = hit ? rihi[q + d] : c;
      }
      rii[q] = a;
      rilo[q] = b;
      rihi[q] = c;
    }
    rifrom = drop >= 4 ? 0u : (rifrom >> (8 * drop));
    riack = drop >= 4 ? 0u : (riack >> (8 * drop));
    ric -= drop;
  }
  // handleLeaderHeartbeatResp (raft.go:1229-1240) for a caught-up remote
  GT_HD void heartbeat_resp(int j, uint64_t clo, uint64_t chi) {
    if (!ract[j]) {
      ract[j] = 1;
      sdirty |= 1u << j;
    }
    if (rst[j] == GR_WAIT) {  // waitToRetry
      rst[j] = GR_RETRY;
      sdirty |= 1u << j;
    }
    GT_BAIL(match[j] < hi);  // sendReplicateMessage: general lane
    if (clo != 0) ri_confirm(clo, chi, (uint32_t)j);
  }
  // handleLeaderReadIndex (raft.go:1171-1203) for a local request (From = NoNode)
  GT_HD void read_index(uint64_t clo, uint64_t chi) {
    if (quorum() == 1) {  // single-voter cluster: ready at once
      add_ready(committed, clo, chi);
      return;
    }
    GT_BAIL(term == 0);
    // hasCommittedEntryAtCurrentTerm: term(committed) from the newest run; with
    // H_GE_LO every index at or above it lies in [firstIndex-1, lastIndex]
    GT_BAIL(!gelo || committed > hi || nruns == 0 || committed < rsn);
    if (rtn != term) return;
    bool dup = false;
#pragma unroll
    for (int q = 0; q < GR_Q; ++q) dup = dup || ((uint32_t)q < ric && rilo[q] == clo && rihi[q] == chi);
    if (!dup) {  // readIndex.addRequest ignores a duplicate context
      uint64_t last = 0;
#pragma unroll
      for (int q = 0; q < GR_Q; ++q) last = ((uint32_t)q + 1 == ric) ? rii[q] : last;
      GT_BAIL(ric > 0 && committed < last);  // index moved backward: panic
      GT_BAIL(ric >= (uint32_t)GR_Q);          // FIFO capacity
      if (!ok) return;
#pragma unroll
      for (int q = 0; q < GR_Q; ++q) {
        const bool hit = (uint32_t)q == ric;
        rii[q] = hit ? committed : rii[q];
        rilo[q] = hit ? clo : rilo[q];
        rihi[q] = hit ? chi : rihi[q];
      }
      rifrom = (rifrom & ~(0xFFu << (8 * ric))) | ((uint32_t)GR_SLOT_NONE << (8 * ric));
      riack &= ~(0xFFu << (8 * ric));
      ric++;
      fifo_dirty = true;
    }
    broadcast_heartbeat(clo, chi);  // also for a duplicate (raft.go:1200-1201)
  }

  // Loads whose need is known only per lane are issued unconditionally, with
  // the address of a line the lane reads anyway (its header) or of one shared
  // line (position 0) when the value is not needed: a branch around a load made
  // the compiler wait for it before the next slot's, so the lane's two rounds of
  // loads became one round trip per slot and message (round 5: 80 vmcnt waits
  // in the S = 5 kernel).
  GT_HD uint64_t ld64(uint32_t row, bool need) const {
    const uint64_t v = kp.st.u64(need ? row : (uint32_t)SR_HDR)[p];
    return need ? v : 0ull;
  }
  GT_HD uint32_t ld8(uint32_t row, bool need) const {
    const uint32_t v = kp.st.u8(row)[need ? p : 0u];
    return need ? v : 0u;
  }

  GT_HD bool step(LaneStats* ls) {
    // ---- round 1: every address is known before any load (routes from the
    // lane index; compile-time route mode)
    uint32_t gin[S];
    routes_of<S, RM>(kp, i, gin, gout);
    uint64_t sw[kTickStageWords] = {};
    if (stage) {
#pragma unroll
      for (uint32_t w = 0; w < kTickStageWords; ++w) sw[w] = stage[w];
    }
    term = s64(SR_TERM);
    committed = s64(SR_COMMITTED);
    hi = s64(SR_LAST_INDEX);
    staged = stage && (uint32_t)(sw[2] >> 32) == kp.pass_tag;
    uint32_t lw = 0, cnt[S], cbs[S];
    if (staged) {  // the steady kernel's loads of this pass (gr_steady.h quiet_step)
      hdr = sw[0];
      etick = sw[1];
      lw = (uint32_t)sw[2];
#pragma unroll
      for (int j = 0; j < S; ++j) cbs[j] = (uint32_t)(sw[3] >> (8 * j)) & 0xFFu;
    } else {
      hdr = s64(SR_HDR);
      etick = s64(SR_ETICK);
      lw = kp.has_locals ? kp.ln.u32(LR_LWORD)[i] : 0u;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const uint32_t c = kp.in.at(gin[j] != NOPOS ? gin[j] : 0u).cnt();
        cbs[j] = gin[j] != NOPOS ? c : 0u;
      }
    }
#pragma unroll
    for (int j = 0; j < S; ++j) {
      outc[j] = 0;
      cnt[j] = mb_n(cbs[j]);
    }
    state = h_state(hdr);
    self = h_self(hdr);
    flags = h_flags(hdr);
    nruns = h_nruns(hdr);
    gelo = h_gelo(hdr);
    tclk[0] = lane_clock(kp);
    uint32_t lf = 0, nt = 0, nq = 0, np = 0;
    if (kp.has_locals) {
      // the packed word holds the whole input when it is ticks and a ReadIndex
      // only (LW_TICKONLY): one row instead of four (gr_layout.h)
      if (lw & LW_TICKONLY) {
        nt = (lw >> LW_TICK_SHIFT) & LW_TICK_MAX;
        lf = (lw & LW_RI) ? LF_READ_INDEX : 0u;
      } else {
        lf = kp.ln.u8(LR_LFLAGS)[i];
        nt = kp.ln.u32(LR_TICKS)[i];
        nq = kp.ln.u32(LR_QTICKS)[i];
        np = kp.ln.u32(LR_PROPOSE)[i];
      }
    }
    const bool leader = state == GR_LEADER;
    GT_BAIL(!leader && state != GR_FOLLOWER);
#pragma unroll
    for (int j = 0; j < S; ++j)  // cold fields lost in the exchange (gr_io.h side_pack): general lane
      GT_BAIL(cnt[j] && !(cbs[j] & MB_UNIFORM) && (cbs[j] & MB_COLD_LOST));
    GT_BAIL((lf & LF_PROPOSE_CC) || nq || np);
    // ---- round 2: one batch of loads, each at a real address when needed
    const bool ri = (lf & LF_READ_INDEX) != 0;
    {
      const uint64_t a = kp.ln.u64(LR_RI_LO)[ri ? i : 0u], b = kp.ln.u64(LR_RI_HI)[ri ? i : 0u];
      rclo = ri ? a : 0ull;
      rchi = ri ? b : 0ull;
    }
    uint64_t retimeout = 0;
    {  // the newest run (the last row): read_index's term test
      const bool nr = nruns && leader && ri;
      rsn = ld64(SR_RUN_START + GR_K - 1, nr);
      rtn = ld64(SR_RUN_TERM + GR_K - 1, nr);
    }
    uint32_t mh[S][MK];
    uint64_t mterm[S][MK], mcom[S][MK], mlo[S][MK], mhi[S][MK];
#pragma unroll
    for (int j = 0; j < S; ++j) {
#pragma unroll
      for (int k = 0; k < MK; ++k) {
        // message k's cold record (tag, term, Commit, Hint, HintHigh: one
        // 64-byte line); a uniform mailbox (Replicates, acks) fails the type
        // test below whatever the record holds
        const bool has = (uint32_t)k < cnt[j];
        const Mailbox mb = kp.in.at(has ? gin[j] : 0u);
        const uint32_t kk = has ? (uint32_t)k : 0u;
        mh[j][k] = mb.tag(kk);
        mterm[j][k] = mb.t32(kk, MT_TERM);
        mcom[j][k] = mb.u64(kk, MF_COMMIT);
        mlo[j][k] = mb.u64(kk, MF_HINT);
        mhi[j][k] = mb.u64(kk, MF_HINT_HIGH);
      }
    }
    htick = ld64(SR_HTICK, leader);
    etimeout = ld64(SR_ETIMEOUT, leader);
    htimeout = ld64(SR_HTIMEOUT, leader);
    retimeout = ld64(SR_RETIMEOUT, !leader);
    ric = leader ? h_ric(hdr) : 0u;
    {
      const uint64_t rb = h_rb(hdr);
#pragma unroll
      for (int j = 0; j < S; ++j) {
        // H_MS: the self slot's MATCH row is stale, its match is lastIndex;
        // H_MP: another slot's is lastIndex - 2
        const bool ms = has_sync_bits(S) && h_ms(hdr) && (uint32_t)j == self;
        const bool mp = has_sync_bits(S) && h_mp(hdr, (uint32_t)j) && (uint32_t)j != self;
        const uint64_t m = ld64(Rw::MATCH + j, leader && !ms && !mp);
        match[j] = ms ? hi : mp ? hi - 2 : m;
        rst[j] = leader ? rb_state(rb, j) : 0u;
        ract[j] = leader ? rb_active(rb, j) : 0u;
        rkind[j] = leader ? rb_kind(rb, j) : 0u;
      }
    }
    // the FIFO's live entries only (entries at or past the count are never
    // read: parity and the host compare the first read_index_count)
#pragma unroll
    for (int q = 0; q < GR_Q; ++q) {
      const bool live = (uint32_t)q < ric;
      rii[q] = ld64(Rw::RI_INDEX + q, live);
      rilo[q] = ld64(Rw::RI_LO + q, live);
      rihi[q] = ld64(Rw::RI_HI + q, live);
      rifrom |= ld8(Rw::B_RIFROM + q, live) << (8 * q);
      riack |= ld8(Rw::B_RIACK + q, live) << (8 * q);
    }
    // every round-2 load is issued before the first value is used: the values
    // pass through an empty asm (keep_value, gr_layout.h), so the optimiser cannot sink the
    // loads under a per-message branch (it did: one wait per message)
#pragma unroll
    for (int j = 0; j < S; ++j) {
#pragma unroll
      for (int k = 0; k < MK; ++k) {
        const bool has = (uint32_t)k < cnt[j];
        const uint32_t tg = keep_value(mh[j][k]);
        const uint64_t tm = keep_value(mterm[j][k]), cm = keep_value(mcom[j][k]);
        const uint64_t lo = keep_value(mlo[j][k]), hh = keep_value(mhi[j][k]);
        mh[j][k] = has ? ((cbs[j] & MB_UNIFORM) ? Mailbox::uniform_tag(cbs[j], k) : tg) & 0xFFu : 0u;
        mterm[j][k] = has ? tm : 0ull;
        mcom[j][k] = has && !leader ? cm : 0ull;
        mlo[j][k] = has ? lo : 0ull;
        mhi[j][k] = has ? hh : 0ull;
      }
    }
    tclk[1] = lane_clock(kp);
    committed0 = committed;
    etick0 = etick;
    htick0 = htick;
    // ---- messages (node.handleReceivedMessages order: slot, then arrival)
#pragma unroll
    for (int j = 0; j < S; ++j) {
      GT_BAIL(cnt[j] > (uint32_t)MK);
#pragma unroll
      for (int k = 0; k < MK; ++k)
        if ((uint32_t)k < cnt[j])
          GT_BAIL(mterm[j][k] != term ||
                  mh[j][k] != (uint32_t)(leader ? GR_HEARTBEAT_RESP : GR_HEARTBEAT));
    }
    uint32_t L = 0, nsrc = 0;
    if (leader) {
      GT_BAIL(flags & F_LTT);  // leader transfer
      GT_BAIL(nt > 1);
#pragma unroll
      for (int j = 0; j < S; ++j) {
#pragma unroll
        for (int k = 0; k < MK; ++k) {
          if ((uint32_t)k < cnt[j]) {
            nmi++;
            if (rkind[j] != GR_SLOT_EMPTY) heartbeat_resp(j, mlo[j][k], mhi[j][k]);
          }
        }
      }
      if (lf & LF_READ_INDEX) read_index(rclo, rchi);
      if (nt) {  // leaderTick (raft.go:403-429)
        etick++;
        if (etick >= etimeout) {
          etick = 0;
          if (flags & GR_F_CHECK_QUORUM) {  // leaderHasQuorum (raft.go:262-271)
            int c = 0;
#pragma unroll
            for (int j = 0; j < S; ++j) {
              if (rkind[j] == GR_SLOT_VOTER && ((uint32_t)j == self || ract[j])) {
                c++;
                if (ract[j]) {
                  ract[j] = 0;
                  sdirty |= 1u << j;
                }
              }
            }
            GT_BAIL(c < quorum());  // step down: general lane
          }
        }
        htick++;
        if (htick >= htimeout) {
          htick = 0;
          uint64_t clo = 0, chi = 0;
#pragma unroll
          for (int q = 0; q < GR_Q; ++q) {
            clo = ((uint32_t)q + 1 == ric) ? rilo[q] : clo;
            chi = ((uint32_t)q + 1 == ric) ? rihi[q] : chi;
          }
          broadcast_heartbeat(clo, chi);
        }
      }
    } else {
      GT_BAIL(lf & LF_READ_INDEX);  // forwarded to the leader: general lane
#pragma unroll
      for (int j = 0; j < S; ++j)
        if (cnt[j]) {
          L = (uint32_t)j;
          nsrc++;
        }
      GT_BAIL(nsrc > 1);
#pragma unroll
      for (int j = 0; j < S; ++j) {
#pragma unroll
        for (int k = 0; k < MK; ++k) {
          if ((uint32_t)k < cnt[j]) {
            nmi++;
            etick = 0;
            if (mcom[j][k] > committed) {  // commitTo (logentry.go:314-323)
              GT_BAIL(mcom[j][k] > hi);
              committed = mcom[j][k];
            }
            emit(j, GR_HEARTBEAT_RESP, 0, mlo[j][k], mhi[j][k]);
          }
        }
      }
      // nonLeaderTick x nt: an election timeout (or the selfRemoved test) goes to the general lane
      GT_BAIL(nt > 0 && etick + nt >= retimeout);
      etick += nt;
    }
    if (!ok) return false;
    // ---- stores
    if (committed != committed0) s64(SR_COMMITTED) = committed;
    uint32_t nf = flags;
    if (etick != etick0) {
      s64(SR_ETICK) = etick;
      nf = (nf & ~F_ETZ) | (etick == 0 ? F_ETZ : 0u);
    }
    if (!leader && nsrc && ((flags & F_LSLOT) >> F_LSLOT_SHIFT) != L + 1) {
      s64(SR_LEADER_ID) = s64(Rw::RID + L);  // setLeaderID(m.From)
      nf = (nf & ~F_LSLOT) | ((L + 1) << F_LSLOT_SHIFT);
    }
    uint64_t nh = (hdr & ~(0xFFull << H_FLAGS_SHIFT)) | ((uint64_t)nf << H_FLAGS_SHIFT);
    if (leader) {
      if (htick != htick0) s64(SR_HTICK) = htick;
      uint64_t rb = h_rb(nh);
#pragma unroll
      for (int j = 0; j < S; ++j) {
        if ((sdirty >> j) & 1u) {
          rb = rb_with(rb, j, 0, 2, rst[j]);
          rb = rb_with(rb, j, 2, 1, ract[j]);
        }
      }
      nh = h_make(state, self, nruns, gelo, nf, fifo_dirty ? ric : h_ric(hdr), rb);
      if (fifo_dirty) {
#pragma unroll
        for (int q = 0; q < GR_Q; ++q) {
          if ((uint32_t)q < ric) {  // the live entries after the pass
            s64(Rw::RI_INDEX + q) = rii[q];
            s64(Rw::RI_LO + q) = rilo[q];
            s64(Rw::RI_HI + q) = rihi[q];
            s8(Rw::B_RIFROM + q) = (uint8_t)(rifrom >> (8 * q));
            s8(Rw::B_RIACK + q) = (uint8_t)(riack >> (8 * q));
          }
        }
      }
    }
    if (nh != hdr) s64(SR_HDR) = nh;
#pragma unroll
    for (int j = 0; j < S; ++j)
      if (gout[j] != NOPOS && (outc[j] || !staged)) kp.out.at(gout[j]).cnt() = (uint8_t)outc[j];
    uint8_t rf = 0;
    if (rtrc) {
      rf |= RF_READY;
      kp.ln.u8(LR_RTR_COUNT)[i] = (uint8_t)rtrc;
#pragma unroll
      for (int q = 0; q < GR_Q; ++q) {
        if ((uint32_t)q < rtrc) {
          kp.ln.u64(LR_RTR_INDEX + q)[i] = rdi[q];
          kp.ln.u64(LR_RTR_LO + q)[i] = rdl[q];
          kp.ln.u64(LR_RTR_HI + q)[i] = rdh[q];
        }
      }
    }
    kp.ln.u8(LR_RFLAGS)[i] = rf;
    tclk[2] = lane_clock(kp);
    const bool adv = committed > committed0;
    ls->leader_commit = adv && leader;
    ls->follower_commit = adv && !leader;
    ls->msgs_in = nmi;
    ls->msgs_out = nmo;
    ls->leader_in = leader ? nmi : 0;
    ls->leader_out = leader ? nmo : 0;
    if (leader) GR_COVER(TICKLANE_LEADER);
    else GR_COVER(TICKLANE_FOLLOWER);
    return true;
  }
};

template <int S, int RM = RM_ANY>
GT_HD bool tick_step(const StepParams& kp, uint32_t i, uint32_t p, LaneStats* ls, const uint64_t* stage = nullptr,
                     uint64_t* clk = nullptr) {
  TickLane<S, RM> L(kp, i, p, stage);
  const bool ok = L.step(ls);
  if (clk) {
    clk[0] = L.tclk[0];
    clk[1] = L.tclk[1];
    clk[2] = L.tclk[2];
  }
  return ok;
}

}  // namespace gr
