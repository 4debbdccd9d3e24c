// gr_lane.h — one Raft group (peer) per lane: the batched restatement of the
// dragonboat raft step (internal/raft) for the HIP kernel in gr_engine.hip.
//
// Each lane owns one engine slot. It loads the slot's state lazily (field
// groups, only what its inputs touch), processes its inputs in the order
// node.handleReceivedMessages / handleEvents gives them (node.go:652-780):
//   messages (remote slot 0..S-1, then arrival order) -> batched ReadIndex ->
//   ticks -> quiesced ticks (one item) -> ProposeEntries,
// and stores back only dirty fields. Anything outside the device fast path
// returns an escalation code; the kernel then re-runs the lane on its pristine
// state up to the escalating item, so every item is applied either entirely on
// the device or entirely by the host (one source of truth).
//
// Function-level citations are to /root/reference/internal/raft/*.go.
#pragma once
#include "gr_cover.h"
#include "gr_layout.h"

namespace gr {

#define GR_HD __host__ __device__ inline __attribute__((always_inline))
#define GR_TRY(x)            \
  do {                       \
    int _e = (x);            \
    if (_e) return _e;       \
  } while (0)

// field groups (lazy load)
enum : uint32_t {
  G_CORE = 1u << 0,   // state flags self term committed last_index
  G_ETICK = 1u << 1,  // electionTick
  G_TICKS = 1u << 2,  // heartbeatTick + the three timeouts
  G_LID = 1u << 3,    // leader_id
  G_LTT = 1u << 4,    // leaderTransferTarget
  G_LEAD = 1u << 5,   // applied node_id
  G_WIN = 1u << 6,    // lo, n_runs, runs
  G_REM = 1u << 7,    // remotes: match next state active kind
  G_SNAP = 1u << 8,   // remotes: snapshotIndex
  G_RI = 1u << 9,     // ReadIndex FIFO
  G_EUB = 1u << 10,   // entry_size_ub
  G_INMEM = 1u << 11, // inMemory.markerIndex / savedTo (truncating merges only)
  G_TICK = G_ETICK | G_TICKS,
};
// dirty bits (store)
enum : uint32_t {
  D_TERM = 1u << 0, D_VOTE = 1u << 1, D_COMMITTED = 1u << 2, D_HI = 1u << 3,
  D_LEADER = 1u << 4, D_LTT = 1u << 5, D_ETICK = 1u << 6, D_HTICK = 1u << 7,
  D_RETIMEOUT = 1u << 8, D_STATE = 1u << 9, D_FLAGS = 1u << 10, D_WIN = 1u << 11,
  D_REM = 1u << 12, D_SNAP = 1u << 13, D_RI = 1u << 14, D_INMEM = 1u << 15,
};

GR_HD bool is_leader_message(uint32_t t) {  // raft.go:986-989
  return t == GR_REPLICATE || t == GR_INSTALL_SNAPSHOT || t == GR_HEARTBEAT ||
         t == GR_TIMEOUT_NOW || t == GR_READ_INDEX_RESP;
}
GR_HD bool is_request_message(uint32_t t) { return t == GR_PROPOSE || t == GR_READ_INDEX; }  // raft.go:982-984
GR_HD uint64_t umin(uint64_t a, uint64_t b) { return a < b ? a : b; }
GR_HD uint64_t umax(uint64_t a, uint64_t b) { return a > b ? a : b; }
GR_HD int popc8(uint32_t x) {
  x &= 0xFFu;
  x = x - ((x >> 1) & 0x55u);
  x = (x & 0x33u) + ((x >> 2) & 0x33u);
  return (int)((x + (x >> 4)) & 0x0Fu);
}

struct OutMsg {
  uint8_t type = 0, flags = 0;
  uint32_t n = 0, run2 = 0;
  uint64_t term = 0, log_index = 0, log_term = 0, commit = 0, hint = 0, hint_high = 0, rt0 = 0, rt1 = 0;
};

struct InMsg {
  uint8_t type, flags;
  uint32_t n, run2;
  uint64_t term, log_index, log_term, commit, hint, hint_high, rt0, rt1;
};

// Per-slot small fields packed 5 bits per slot (state, active, kind): rb_* in gr_layout.h.

// The general lane: every handler of the device path. The steady-state
// subset runs first in the lean lane of gr_fast.h; this lane steps the lanes
// that one hands over.
template <int S>
struct Lane {
  using R = Rows<S>;
  const StepParams kp;  // by value: small, uniform (SGPRs)
  const uint32_t p;     // engine slot (state rows)
  const uint32_t i;     // lane (per-pass rows)
  uint32_t loaded = 0, dirty = 0;

  // G_CORE
  uint64_t hdr0 = 0;  // the header word as loaded
  uint64_t hi_ld = 0;  // lastIndex as loaded (the sync bits' reference, gr_layout.h)
  uint32_t state = 0, flags = 0, self = GR_SLOT_NONE;
  uint64_t term = 0, committed = 0, hi = 0;
  // G_ETICK / G_TICKS
  uint64_t etick = 0, htick = 0, retimeout = 0, etimeout = 0, htimeout = 0;
  // G_LID / G_LTT / G_LEAD
  uint64_t leader_id = 0, ltt = 0, applied = 0, node_id = 0;
  // G_WIN
  uint64_t lo = 0;
  uint32_t nruns = 0;
  uint64_t rs[GR_K], rt[GR_K];
  // G_REM / G_SNAP
  uint64_t match[S], next[S], snap[S];
  uint64_t rb = 0;
  uint32_t snapz = 0;  // slots whose snapshotIndex is reset to 0 without a load
  // G_RI
  uint32_t ric = 0, rifrom = 0, riack = 0;  // from/ack: one byte per FIFO entry
  uint64_t rii[GR_Q], rilo[GR_Q], rihi[GR_Q];
  // G_EUB
  uint64_t eub = 0;
  // G_INMEM
  uint64_t imk = 0, isv = 0;  // inMemory.markerIndex, savedTo

  // outputs of this pass
  uint64_t tclk[3] = {0, 0, 0};  // GR_WAVE_CLOCK phase marks (device builds): loads, run, store done
  uint32_t outcnt = 0;  // 3 bits per slot
  uint64_t outu = 0;    // 5 bits per slot: not uniform, ReplicateResp kind, MB_N1 of messages 0..2
  uint32_t rtrc = 0, prop_result = 0;
  bool rand_used = false;
  uint64_t append_from = 0, propose_first = 0;
  uint32_t fwd_n = 0, fwd_entries = 0;  // forwarded Propose batches appended this pass
  uint64_t committed0 = 0;
  uint32_t msgs_in = 0, msgs_out = 0, entries_in = 0;


  // The general kernel's message prefetch (round 5, device builds, S <= 3): the
  // first kPfK messages of every in-mailbox, loaded before the message loop by
  // LDS-DMA (global_load_lds) into this wave's region of the kernel's LDS, so the
  // loop reads them there instead of making one dependent round of global loads
  // per message (GR_WAVE_CLOCK, round 4: the loop was 85-110 us of a config-5
  // wave's 60-200). Per message: the 64-byte cold record as 4 x 16 B, then
  // LogIndex low, high, Commit offset and the term word as 4 x 4 B; each piece
  // is one wave-instruction (64 lanes, lane-linear). pf_ = nullptr: no prefetch.
  static constexpr uint32_t kPfK = 2, kPfRec = 4 * 64 * 16, kPfBytes = kPfRec + 4 * 64 * 4;
  static constexpr uint32_t kPfWave = S <= 3 ? (uint32_t)S * kPfK * kPfBytes : 0u;
  uint8_t* pf_ = nullptr;

  GR_HD Lane(const StepParams& k, uint32_t lane, uint32_t peer) : kp(k), p(peer), i(lane) {}

  GR_HD uint64_t& s64(uint32_t row) const { return kp.st.u64(row)[p]; }
  GR_HD uint8_t& s8(uint32_t row) const { return kp.st.u8(row)[p]; }

  // ---------------------------------------------------------------- loading
  GR_HD void need(uint32_t g) {
    if (g & (G_WIN | G_REM | G_RI)) g |= G_CORE;  // their small fields live in the header word
    const uint32_t miss = g & ~loaded;
    if (!miss) return;
    if (miss & G_CORE) {
      hdr0 = s64(SR_HDR);
      state = h_state(hdr0);
      flags = h_flags(hdr0);
      self = h_self(hdr0);
      term = s64(SR_TERM);
      committed = s64(SR_COMMITTED);
      committed0 = committed;
      hi = s64(SR_LAST_INDEX);
      hi_ld = hi;
    }
    if (miss & G_ETICK) etick = s64(SR_ETICK);
    if (miss & G_LID) leader_id = s64(SR_LEADER_ID);
    if (miss & G_LTT) ltt = s64(SR_LTT);
    if (miss & G_TICKS) {
      htick = s64(SR_HTICK);
      retimeout = s64(SR_RETIMEOUT);
      etimeout = s64(SR_ETIMEOUT);
      htimeout = s64(SR_HTIMEOUT);
    }
    if (miss & G_LEAD) {
      applied = s64(SR_APPLIED);
      node_id = s64(SR_NODE_ID);
    }
    if (miss & G_WIN) {
      lo = s64(SR_LO);
      nruns = h_nruns(hdr0);
      if (nruns > GR_K) nruns = GR_K;
#pragma unroll
      for (int r = 0; r < GR_K; ++r) {  // right-aligned rows -> oldest-first registers
        const bool v = (uint32_t)r < nruns;
        rs[r] = v ? s64(SR_RUN_START + run_row(nruns, r)) : 0;
        rt[r] = v ? s64(SR_RUN_TERM + run_row(nruns, r)) : 0;
      }
    }
    if (miss & G_REM) {
      rb = h_rb(hdr0) & ((1ull << (5 * S)) - 1);
      const uint64_t sb = has_sync_bits(S) ? hdr0 : 0;  // stale rows: values from lastIndex as loaded
#pragma unroll
      for (int j = 0; j < S; ++j) {
        match[j] = (h_ms(sb) && (uint32_t)j == h_self(hdr0))  ? hi_ld
                   : (h_mp(sb, (uint32_t)j) && (uint32_t)j != h_self(hdr0)) ? hi_ld - 2
                                                                          : s64(R::MATCH + j);
        next[j] = h_nx(sb, (uint32_t)j) ? hi_ld + 1 : s64(R::NEXT + j);
      }
    }
    if (miss & G_SNAP) {
#pragma unroll
      for (int j = 0; j < S; ++j) snap[j] = ((snapz >> j) & 1u) ? 0 : s64(R::SNAP + j);
    }
    if (miss & G_RI) {
      ric = h_ric(hdr0);
      rifrom = 0;
      riack = 0;
#pragma unroll
      for (int q = 0; q < GR_Q; ++q) {
        rii[q] = s64(R::RI_INDEX + q);
        rilo[q] = s64(R::RI_LO + q);
        rihi[q] = s64(R::RI_HI + q);
        rifrom |= (uint32_t)s8(R::B_RIFROM + q) << (8 * q);
        riack |= (uint32_t)s8(R::B_RIACK + q) << (8 * q);
      }
    }
    if (miss & G_EUB) eub = s64(SR_ENTRY_UB);
    if (miss & G_INMEM) {
      imk = s64(SR_MARKER);
      isv = s64(SR_SAVED_TO);
    }
    loaded |= miss;
  }


  GR_HD void store() {
    // Sync bits (gr_layout.h) hold only while lastIndex and the remote rows do:
    // a pass that changes either writes the remote rows out and clears them.
    const bool unsync = has_sync_bits(S) && (hdr0 & H_SYNC_MASK) && (dirty & (D_HI | D_REM));
    if (unsync) {
      need(G_REM);
      dirty |= D_REM;
    }
    if (dirty & (D_LTT | D_ETICK | D_LEADER)) {  // device-internal flag bits (gr_layout.h)
      need(G_CORE);
      uint32_t nf = flags;
      if (dirty & D_LTT) nf = (nf & ~F_LTT) | (ltt ? F_LTT : 0u);
      if (dirty & D_ETICK) nf = (nf & ~F_ETZ) | (etick == 0 ? F_ETZ : 0u);
      if (dirty & D_LEADER) {
        uint32_t sl = 0;
#pragma unroll 1
        for (uint32_t j = 0; j < (uint32_t)S && j < 7 && leader_id; ++j)
          if (!sl && remote_id(j) == leader_id) sl = j + 1;
        nf = (nf & ~F_LSLOT) | (sl << F_LSLOT_SHIFT);
      }
      if (nf != flags) {
        flags = nf;
        dirty |= D_FLAGS;
      }
    }
    if (dirty & D_TERM) s64(SR_TERM) = term;
    if (dirty & D_VOTE) s64(SR_VOTE) = 0;  // reset() on a term change is the only vote write here
    if (dirty & D_COMMITTED) s64(SR_COMMITTED) = committed;
    if (dirty & D_HI) s64(SR_LAST_INDEX) = hi;
    if (dirty & D_LEADER) s64(SR_LEADER_ID) = leader_id;
    if (dirty & D_LTT) s64(SR_LTT) = ltt;
    if (dirty & D_ETICK) s64(SR_ETICK) = etick;
    if (dirty & D_HTICK) s64(SR_HTICK) = htick;
    if (dirty & D_RETIMEOUT) s64(SR_RETIMEOUT) = retimeout;
    if (dirty & D_INMEM) {
      s64(SR_MARKER) = imk;
      s64(SR_SAVED_TO) = isv;
    }
    if (dirty & D_WIN) {
#pragma unroll
      for (int r = 0; r < GR_K; ++r) {  // oldest-first registers -> right-aligned rows
        if ((uint32_t)r < nruns) {
          s64(SR_RUN_START + run_row(nruns, r)) = rs[r];
          s64(SR_RUN_TERM + run_row(nruns, r)) = rt[r];
        }
      }
    }
    if (dirty & D_REM) {
#pragma unroll
      for (int j = 0; j < S; ++j) {
        s64(R::MATCH + j) = match[j];
        s64(R::NEXT + j) = next[j];
      }
    }
    if (dirty & D_SNAP) {
#pragma unroll
      for (int j = 0; j < S; ++j) s64(R::SNAP + j) = snap[j];
    } else if (snapz) {
#pragma unroll
      for (int j = 0; j < S; ++j)
        if ((snapz >> j) & 1u) s64(R::SNAP + j) = 0;
    }
    if (dirty & D_RI) {  // the live entries only: nothing reads past the count (gr_tick.h, parity)
#pragma unroll
      for (int q = 0; q < GR_Q; ++q) {
        if ((uint32_t)q < ric) {
          s64(R::RI_INDEX + q) = rii[q];
          s64(R::RI_LO + q) = rilo[q];
          s64(R::RI_HI + q) = rihi[q];
          s8(R::B_RIFROM + q) = (uint8_t)(rifrom >> (8 * q));
          s8(R::B_RIACK + q) = (uint8_t)(riack >> (8 * q));
        }
      }
    }
    // one header word for the small fields; the run bits follow term, committed
    // and the window (gr_layout.h)
    const uint32_t hdr_dirty = D_STATE | D_FLAGS | D_WIN | D_REM | D_RI |
                               (has_run_bits(S) ? (D_TERM | D_COMMITTED | D_HI) : 0u);
    if (dirty & hdr_dirty) {
      uint64_t h = hdr0;
      const uint64_t remmask = ((1ull << (5 * S)) - 1) << H_REM_SHIFT;
      const uint64_t keep_rem = h & (~0ull << H_REM_SHIFT) & ~remmask & ~(unsync ? H_SYNC_MASK : 0ull);
      uint32_t nr = h_nruns(h);
      bool gelo = h_gelo(h);
      if (dirty & D_WIN) {
        uint64_t last_start = 0;
#pragma unroll
        for (int r = 0; r < GR_K; ++r) last_start = ((uint32_t)r + 1 == nruns) ? rs[r] : last_start;
        nr = nruns;
        gelo = nruns && last_start >= lo;
      }
      const uint64_t rbits = (dirty & D_REM) ? rb : (h_rb(h) & ((1ull << (5 * S)) - 1));
      h = h_make(state, self, nr, gelo, flags, (dirty & D_RI) ? ric : h_ric(h), 0) | keep_rem |
          (rbits << H_REM_SHIFT);
      if (has_run_bits(S)) {
        h &= ~H_RUN_MASK;
        if (loaded & G_WIN) {
          uint64_t ns = 0, nt = 0;
#pragma unroll
          for (int r = 0; r < GR_K; ++r) {
            ns = ((uint32_t)r + 1 == nruns) ? rs[r] : ns;
            nt = ((uint32_t)r + 1 == nruns) ? rt[r] : nt;
          }
          h |= run_bits(nruns, ns, nt, term, committed);
        }  // else: cleared (the window was not read)
      }
      if (h != hdr0) s64(SR_HDR) = h;
    }
  }

  // write-only updates (no load needed)
  GR_HD void zero_etick() {
    etick = 0;
    loaded |= G_ETICK;
    dirty |= D_ETICK;
  }
  GR_HD void zero_snap(uint32_t j) {  // remote.reset(), remote.go:61-63
    if (loaded & G_SNAP) {
      put(snap, j, (uint64_t)0);
      dirty |= D_SNAP;
    } else {
      snapz |= 1u << j;
    }
  }

  // runtime-slot access to register arrays (unrolled selects; no scratch)
  template <typename T, int N>
  GR_HD T sel(const T (&a)[N], uint32_t j) const {
    // mask-and-or, not a select chain: LLVM folds selects of adjacent loads
    // back into a dynamically indexed load, which pins the lane in scratch.
    uint64_t v = 0;
#pragma unroll
    for (int x = 0; x < N; ++x) v |= (uint64_t)a[x] & (0ull - (uint64_t)((uint32_t)x == j));
    return (T)v;
  }
  template <typename T, int N>
  GR_HD void put(T (&a)[N], uint32_t j, T v) {
#pragma unroll
    for (int x = 0; x < N; ++x) {
      const uint64_t m = 0ull - (uint64_t)((uint32_t)x == j);
      a[x] = (T)(((uint64_t)a[x] & ~m) | ((uint64_t)v & m));
    }
  }
  GR_HD uint32_t rstate(uint32_t j) const { return rb_state(rb, j); }
  GR_HD uint32_t rkind(uint32_t j) const { return rb_kind(rb, j); }
  GR_HD uint32_t ractive(uint32_t j) const { return rb_active(rb, j); }
  GR_HD void set_rstate(uint32_t j, uint32_t v) { rb = rb_with(rb, j, 0, 2, v); }
  GR_HD void set_ractive(uint32_t j, uint32_t v) { rb = rb_with(rb, j, 2, 1, v); }

  GR_HD uint64_t remote_id(uint32_t j) const { return s64(R::RID + j); }
  GR_HD uint32_t find_slot(uint64_t id) {  // node id -> slot, NONE if not a member
    need(G_REM);
    uint32_t s = GR_SLOT_NONE;
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)S; ++j)
      if (rkind(j) != GR_SLOT_EMPTY && remote_id(j) == id) s = j;
    return s;
  }

  // ---------------------------------------------------------------- quorum
  GR_HD int voters() {
    need(G_REM);
    int nv = 0;
#pragma unroll
    for (int j = 0; j < S; ++j) nv += rkind(j) == GR_SLOT_VOTER;
    return nv;
  }
  GR_HD int quorum() { return voters() / 2 + 1; }  // raft.go:254-256
  GR_HD bool self_removed() {                      // raft.go:813-820
    need(G_CORE | G_REM);
    if (self >= (uint32_t)S) return true;
    const uint32_t k = rkind(self);
    return state == GR_OBSERVER ? k != GR_SLOT_OBSERVER : k != GR_SLOT_VOTER;
  }

  // ---------------------------------------------------------------- log window
  // entryLog.term (logentry.go:141-157) over the device term-run window.
  GR_HD int term_of(uint64_t x, uint64_t* t) {
    need(G_CORE | G_WIN);
    if (x < lo || x > hi) { *t = 0; return 0; }
    if (nruns == 0 || x < rs[0]) return GR_ESC_TERM_WINDOW;
    uint64_t v = rt[0];
#pragma unroll
    for (int r = 1; r < GR_K; ++r) v = ((uint32_t)r < nruns && rs[r] <= x) ? rt[r] : v;
    *t = v;
    return 0;
  }
  GR_HD uint64_t last_run_term() const {
    uint64_t v = 0;
#pragma unroll
    for (int r = 0; r < GR_K; ++r) v = ((uint32_t)r + 1 == nruns) ? rt[r] : v;
    return v;
  }
  // append a run starting at `start` with term t (extends the last run when
  // the term is unchanged; drops the oldest run when the window is full).
  GR_HD void win_push(uint64_t start, uint64_t t) {
    if (nruns > 0 && last_run_term() == t) return;
    if (nruns < GR_K) {
#pragma unroll
      for (int r = 0; r < GR_K; ++r) {
        const bool hit = (uint32_t)r == nruns;
        rs[r] = hit ? start : rs[r];
        rt[r] = hit ? t : rt[r];
      }
      nruns++;
    } else {
#pragma unroll
      for (int r = 0; r + 1 < GR_K; ++r) { rs[r] = rs[r + 1]; rt[r] = rt[r + 1]; }
      rs[GR_K - 1] = start;
      rt[GR_K - 1] = t;
    }
    dirty |= D_WIN;
  }
  GR_HD void win_truncate(uint64_t ci) {  // drop runs starting at >= ci
    uint32_t n = 0;
#pragma unroll
    for (int r = 0; r < GR_K; ++r) n = ((uint32_t)r < nruns && rs[r] < ci) ? (uint32_t)(r + 1) : n;
    if (n != nruns) { nruns = n; dirty |= D_WIN; }
  }

  // ---------------------------------------------------------------- remotes (remote.go)
  GR_HD bool is_paused(uint32_t s) const { return s == GR_WAIT || s == GR_SNAPSHOT_ST; }  // :158-171
  GR_HD void wait_to_retry(uint32_t j) {  // :81-85
    if (rstate(j) == GR_WAIT) set_rstate(j, GR_RETRY);
  }
  GR_HD void become_retry(uint32_t j) {  // :65-73
    const uint64_t m = sel(match, j);
    uint64_t nx = m + 1;
    if (rstate(j) == GR_SNAPSHOT_ST) {
      need(G_SNAP);
      nx = umax(m + 1, sel(snap, j) + 1);
    }
    put(next, j, nx);
    zero_snap(j);
    set_rstate(j, GR_RETRY);
  }
  GR_HD void become_replicate(uint32_t j) {  // :92-96
    put(next, j, sel(match, j) + 1);
    zero_snap(j);
    set_rstate(j, GR_REPLICATE_ST);
  }
  GR_HD void responded_to(uint32_t j) {  // :130-138
    const uint32_t s = rstate(j);
    if (s == GR_RETRY) {
      GR_COVER(RESPONDED_RETRY);
      become_replicate(j);
    } else if (s == GR_SNAPSHOT_ST) {
      need(G_SNAP);
      if (sel(match, j) >= sel(snap, j)) {
        GR_COVER(RESPONDED_SNAPSHOT_RETRY);
        become_retry(j);
      } else {
        GR_COVER(RESPONDED_SNAPSHOT_STAY);
      }
    }
  }
  GR_HD bool try_update(uint32_t j, uint64_t index) {  // :108-118
    if (sel(next, j) < index + 1) put(next, j, index + 1);
    if (sel(match, j) < index) {
      wait_to_retry(j);
      put(match, j, index);
      return true;
    }
    return false;
  }
  GR_HD bool decrease_to(uint32_t j, uint64_t rejected, uint64_t last) {  // :140-156
    if (rstate(j) == GR_REPLICATE_ST) {
      if (rejected <= sel(match, j)) {
        GR_COVER(DECREASE_IGNORED);
        return false;
      }
      GR_COVER(DECREASE_REPLICATE);
      put(next, j, sel(match, j) + 1);
      return true;
    }
    if (sel(next, j) - 1 != rejected) {
      GR_COVER(DECREASE_IGNORED);
      return false;
    }
    GR_COVER(DECREASE_PROBE);
    wait_to_retry(j);
    put(next, j, umax(1, umin(rejected, last + 1)));
    return true;
  }
  GR_HD void enter_retry(uint32_t j) {  // raft.go:1307-1311
    if (rstate(j) == GR_REPLICATE_ST) become_retry(j);
  }

  // ---------------------------------------------------------------- emission
  // routes, mailbox count bytes and local inputs, read once per pass in the
  // first load round (preload): the message and local-input loops then start
  // without a dependent load round per slot
  // GR_LANE_PRELOAD=0 (A/B builds): routes and counts computed or loaded where
  // they are used instead (fewer live registers across the message loop: 72 B
  // of scratch instead of 128, but config 5's general kernel measured 178 vs
  // 173 us per pass, the setup round saved and more dependent rounds in the loop)
#ifndef GR_LANE_PRELOAD
#define GR_LANE_PRELOAD 1
#endif
  uint32_t gin_[S], gout_[S], pcb_[S];
  uint32_t plf_ = 0, pnt_ = 0, pnq_ = 0, pnp_ = 0;
  GR_HD void preload() {
    if (!GR_LANE_PRELOAD) return;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      gin_[j] = route_of(kp, 0, (uint32_t)j, i);
      gout_[j] = route_of(kp, 1, (uint32_t)j, i);
    }
#pragma unroll
    for (int j = 0; j < S; ++j) pcb_[j] = gin_[j] != NOPOS ? (uint32_t)kp.in.at(gin_[j]).cnt() : 0u;
    if (kp.has_locals) {
      plf_ = kp.ln.u8(LR_LFLAGS)[i];
      pnt_ = kp.ln.u32(LR_TICKS)[i];
      pnq_ = kp.ln.u32(LR_QTICKS)[i];
      pnp_ = kp.ln.u32(LR_PROPOSE)[i];
    }
  }
  // Issue the message prefetch (pf_): every piece of every (slot, message) pair
  // below kPfK, at its address when the mailbox holds that message (the cold
  // record only for a mailbox without MB_UNIFORM), else at position 0's (one
  // shared line). Needs preload()'s routes and count bytes.
  GR_HD void prefetch() {
#if defined(__HIP_DEVICE_COMPILE__)
    if (!GR_LANE_PRELOAD || kPfWave == 0 || !pf_) return;
    const Mailbox d0 = kp.in.at(0);
#pragma unroll
    for (int j = 0; j < S; ++j) {
#pragma unroll
      for (uint32_t k = 0; k < kPfK; ++k) {
        const uint32_t cb = pcb_[j];
        const bool v = gin_[j] != NOPOS && k < mb_n(cb) && k < kp.in.depth;
        const Mailbox mb = v ? kp.in.at(gin_[j]) : d0;
        const uint32_t kk = v ? k : 0u;
        const bool full = v && !(cb & MB_UNIFORM);
        const uint4* rec = reinterpret_cast<const uint4*>(full ? mb.rec(kk) : d0.rec(0));
        uint8_t* base = pf_ + ((uint32_t)j * kPfK + k) * kPfBytes;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) __builtin_amdgcn_global_load_lds((const void*)(rec + q), (void*)(base + q * 1024), 16, 0, 0);
        const uint32_t* li = reinterpret_cast<const uint32_t*>(&mb.u64(kk, MF_LOG_INDEX));
        __builtin_amdgcn_global_load_lds((const void*)li, (void*)(base + kPfRec), 4, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)(li + 1), (void*)(base + kPfRec + 256), 4, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)&mb.t32(kk, MT_CDELTA), (void*)(base + kPfRec + 512), 4, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)&mb.mterm(), (void*)(base + kPfRec + 768), 4, 0, 0);
      }
    }
#endif
  }
  GR_HD uint32_t out_gpos(uint32_t j) const { return GR_LANE_PRELOAD ? sel(gout_, j) : route_of(kp, 1, j, i); }
  GR_HD uint32_t in_gpos(uint32_t j) const { return GR_LANE_PRELOAD ? sel(gin_, j) : route_of(kp, 0, j, i); }
  // raft.send (raft.go:457-461): From is implied by the mailbox; Term is
  // r.term unless the type is a request (finalizeMessageTerm :444-455).
  GR_HD int emit(uint32_t j, const OutMsg& m) {
    need(G_CORE);
    if (j >= (uint32_t)S) return GR_ESC_NONMEMBER;
    const uint32_t g = out_gpos(j);
    if (g == NOPOS) return GR_ESC_NONMEMBER;
    const uint32_t c = (outcnt >> (3 * j)) & 7u;
    if (c >= kp.out.depth) return GR_ESC_CAPACITY;
    const uint64_t mterm = is_request_message(m.type) ? m.term : term;
    if (wide_term(mterm, m.log_term, m.rt0, m.rt1)) return GR_ESC_WIDE_TERM;
    const Mailbox mb = kp.out.at(g);
    mb.type(c) = m.type;
    mb.flags(c) = m.flags;
    mb.t32(c, MT_TERM) = (uint32_t)mterm;
    switch (m.type) {  // write the fields the receiver reads (read_msg)
      case GR_REPLICATE: {
        mb.n(c) = m.n;
        mb.u64(c, MF_LOG_INDEX) = m.log_index;
        mb.t32(c, MT_LOG_TERM) = (uint32_t)(m.log_term);
        uint32_t cd;
        if (commit_delta(m.commit, m.log_index, &cd)) {
          mb.t32(c, MT_CDELTA) = cd;
        } else {
          mb.flags(c) = (uint8_t)(m.flags | MFL_WIDE_COMMIT);
          mb.u64(c, MF_COMMIT) = m.commit;
        }
        if (m.n) {
          mb.t32(c, MT_RT0) = (uint32_t)(m.rt0);
          if (((m.flags >> MFL_RUNS_SHIFT) & 3u) == 2) {
            mb.run2(c) = m.run2;
            mb.t32(c, MT_RT1) = (uint32_t)(m.rt1);
          }
        }
        break;
      }
      case GR_REPLICATE_RESP:  // Hint is only read on a reject (decreaseTo, raft.go:1219)
        mb.u64(c, MF_LOG_INDEX) = m.log_index;
        if (m.flags & MFL_REJECT) mb.u64(c, MF_HINT) = m.hint;
        break;
      case GR_HEARTBEAT:
        mb.u64(c, MF_COMMIT) = m.commit;
        mb.u64(c, MF_HINT) = m.hint;
        mb.u64(c, MF_HINT_HIGH) = m.hint_high;
        break;
      case GR_HEARTBEAT_RESP:
        mb.u64(c, MF_HINT) = m.hint;
        mb.u64(c, MF_HINT_HIGH) = m.hint_high;
        break;
      default:
        mb.n(c) = m.n;
        mb.run2(c) = m.run2;
        mb.u64(c, MF_LOG_INDEX) = m.log_index;
        mb.t32(c, MT_LOG_TERM) = (uint32_t)(m.log_term);
        mb.u64(c, MF_COMMIT) = m.commit;
        mb.u64(c, MF_HINT) = m.hint;
        mb.u64(c, MF_HINT_HIGH) = m.hint_high;
        mb.t32(c, MT_RT0) = (uint32_t)(m.rt0);
        mb.t32(c, MT_RT1) = (uint32_t)(m.rt1);
        break;
    }
    // uniform mailbox bookkeeping (gr_layout.h MB_UNIFORM): compact Replicates or
    // accepts of one kind and one term, at most kUniformMax; the term word is
    // written with message 0 and compared with it by the later ones
    uint32_t cd0;
    const uint32_t runs = (m.flags >> MFL_RUNS_SHIFT) & 3u;
    const bool resp = m.type == GR_REPLICATE_RESP;
    const bool uni = resp ? !(m.flags & MFL_REJECT)
                          : m.type == GR_REPLICATE && commit_delta(m.commit, m.log_index, &cd0) &&
                                m.log_term == mterm &&
                                (m.n == 0 ? runs == 0 : (m.n == 1 && runs == 1 && m.rt0 == mterm));
    const uint32_t sh = 5 * j;
    if (c == 0) {
      mb.mterm() = (uint32_t)mterm;
      if (resp) outu |= 2ull << sh;
    } else if (mb.mterm() != (uint32_t)mterm || resp != (((outu >> sh) & 2ull) != 0)) {
      outu |= 1ull << sh;
    }
    if (!uni || c >= kUniformMax) outu |= 1ull << sh;
    else if (!resp && m.n) outu |= 4ull << (sh + c);
    outcnt += 1u << (3 * j);
    msgs_out++;
    return 0;
  }
  GR_HD int add_ready(uint64_t index, uint64_t clo, uint64_t chi) {  // raft.go:1163-1169
    if (rtrc >= GR_Q) return GR_ESC_CAPACITY;
    kp.ln.u64(LR_RTR_INDEX + rtrc)[i] = index;
    kp.ln.u64(LR_RTR_LO + rtrc)[i] = clo;
    kp.ln.u64(LR_RTR_HI + rtrc)[i] = chi;
    rtrc++;
    return 0;
  }

  // ---------------------------------------------------------------- reset / transitions
  // raft.reset (raft.go:704-720) with the random draw supplied by the host.
  GR_HD int reset(uint64_t t) {
    if (rand_used || !kp.has_locals) return GR_ESC_RANDOM;
    need(G_CORE | G_TICKS | G_REM);
    if (etimeout == 0) return GR_ESC_PANIC;
    rand_used = true;
    const uint64_t rand_value = kp.ln.u64(LR_RAND)[i];
    if (term != t) {
      term = t;
      dirty |= D_TERM | D_VOTE;  // vote = NoLeader
    }
    leader_id = 0;
    loaded |= G_LID;
    etick = 0;
    loaded |= G_ETICK;
    htick = 0;
    retimeout = etimeout + rand_value % etimeout;  // raft.go:435-438
    ric = 0;
    rifrom = 0;
    riack = 0;
#pragma unroll
    for (int q = 0; q < GR_Q; ++q) { rii[q] = 0; rilo[q] = 0; rihi[q] = 0; }
    loaded |= G_RI;
    flags &= ~(uint32_t)GR_F_PENDING_CONFIG_CHANGE;
    ltt = 0;
    loaded |= G_LTT;
#pragma unroll
    for (int j = 0; j < S; ++j) {  // resetRemotes/resetObservers :733-753
      if (rkind(j) != GR_SLOT_EMPTY) {
        next[j] = hi + 1;
        match[j] = (uint32_t)j == self ? hi : 0;
        set_rstate(j, GR_RETRY);
        set_ractive(j, 0);
        zero_snap(j);
      }
    }
    dirty |= D_LEADER | D_ETICK | D_HTICK | D_RETIMEOUT | D_RI | D_FLAGS | D_LTT | D_REM;
    return 0;
  }
  GR_HD int become_follower(uint64_t t, uint64_t lid) {  // raft.go:669-674
    // a step-down after appending forwarded proposals: the host attributes
    // those entries from propose_first, which only holds while this lane leads
    if (fwd_n) return GR_ESC_UNSUPPORTED;
    need(G_CORE);
    state = GR_FOLLOWER;
    dirty |= D_STATE;
    GR_TRY(reset(t));
    leader_id = lid;
    return 0;
  }
  GR_HD int become_observer(uint64_t t, uint64_t lid) {  // raft.go:660-667
    GR_TRY(reset(t));
    leader_id = lid;
    return 0;
  }
  GR_HD void set_leader_from(uint32_t j) {  // setLeaderID(m.From), raft.go:239-244
    leader_id = remote_id(j);
    loaded |= G_LID;
    dirty |= D_LEADER;
  }

  // ---------------------------------------------------------------- commit (kernel step 1)
  // raft.tryCommit + sortMatchValues + entryLog.tryCommit (raft.go:600-641,
  // logentry.go:359-374): order statistic of the voting match values by a
  // compile-time sorting network; non-voters sort to the end as +inf.
  GR_HD int try_commit(bool* out) {
    need(G_CORE | G_REM);
    *out = false;
    uint64_t m[S];
    int nv = 0;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const bool v = rkind(j) == GR_SLOT_VOTER;
      m[j] = v ? match[j] : ~0ull;
      nv += v;
    }
    if (nv == 0) return GR_ESC_PANIC;  // matched[len-quorum] out of range
#pragma unroll
    for (int r = 0; r < S; ++r) {  // odd-even transposition network
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
    if (q <= committed) return 0;
    uint64_t lt;
    GR_TRY(term_of(q, &lt));
    if (lt == term) {
      if (q > hi) return GR_ESC_PANIC;  // commitTo, logentry.go:318-321
      committed = q;
      dirty |= D_COMMITTED;
      *out = true;
    }
    return 0;
  }

  // ---------------------------------------------------------------- replicate (leader side)
  // raft.sendReplicateMessage + makeReplicateMessage (raft.go:474-532).
  GR_HD int send_replicate(uint32_t j) {
    need(G_CORE | G_REM | G_WIN);
    if (is_paused(rstate(j))) {
      GR_COVER(SEND_PAUSED);
      return 0;
    }
    const uint64_t nx = sel(next, j);
    uint64_t lt;
    GR_TRY(term_of(nx - 1, &lt));
    OutMsg m;
    m.type = GR_REPLICATE;
    m.log_index = nx - 1;
    m.log_term = lt;
    m.commit = committed;
    if (nx <= hi) {  // entries(next, maxSize), logentry.go:231-236
      if (nx <= lo) return GR_ESC_SNAPSHOT;  // checkBound -> ErrCompacted
      if (nruns == 0 || nx < rs[0]) return GR_ESC_TERM_WINDOW;
      const uint64_t cnt = hi - nx + 1;
      if (cnt > 0xFFFFFFFFull) return GR_ESC_CAPACITY;
      if (cnt > 1) {  // limitSize (entryutils.go:50-63) keeps all iff sum <= max
        GR_COVER(SEND_MULTI_ENTRY);
        need(G_EUB);
        if (eub == 0 || cnt > kp.max_entry_size / eub) return GR_ESC_ENTRY_SIZE;
      }
      uint32_t r0 = 0;
#pragma unroll
      for (int r = 1; r < GR_K; ++r) r0 = ((uint32_t)r < nruns && rs[r] <= nx) ? (uint32_t)r : r0;
      const uint32_t nr = nruns - r0;
      if (nr > 2) return GR_ESC_MSG_RUNS;
      uint64_t t0 = rt[0], t1 = 0, s1 = 0;
#pragma unroll
      for (int r = 0; r < GR_K; ++r) {
        t0 = ((uint32_t)r == r0) ? rt[r] : t0;
        t1 = ((uint32_t)r == r0 + 1) ? rt[r] : t1;
        s1 = ((uint32_t)r == r0 + 1) ? rs[r] : s1;
      }
      m.n = (uint32_t)cnt;
      m.rt0 = t0;
      if (nr == 2) {
        GR_COVER(SEND_TWO_RUNS);
        m.rt1 = t1;
        m.run2 = (uint32_t)(s1 - nx);
        m.flags = (uint8_t)(2 << MFL_RUNS_SHIFT);
      } else {
        m.flags = (uint8_t)(1 << MFL_RUNS_SHIFT);
      }
      const uint32_t s = rstate(j);  // remote.progress(lastIndex) :120-128
      if (s == GR_REPLICATE_ST) put(next, j, hi + 1);
      else if (s == GR_RETRY) set_rstate(j, GR_WAIT);
      else return GR_ESC_PANIC;
      dirty |= D_REM;
    } else {
      GR_COVER(SEND_EMPTY);
    }
    return emit(j, m);
  }
  GR_HD int broadcast_replicate() {  // raft.go:534-546
    need(G_CORE | G_REM);
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)S; ++j)
      if (rkind(j) == GR_SLOT_VOTER && j != self) GR_TRY(send_replicate(j));
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)S; ++j) {
      if (rkind(j) == GR_SLOT_OBSERVER) {
        if (j == self) return GR_ESC_PANIC;
        GR_COVER(BCAST_OBSERVER);
        GR_TRY(send_replicate(j));
      }
    }
    return 0;
  }
  GR_HD int send_heartbeat(uint32_t j, uint64_t clo, uint64_t chi) {  // raft.go:548-564
    OutMsg m;
    m.type = GR_HEARTBEAT;
    m.commit = umin(sel(match, j), committed);
    m.hint = clo;
    m.hint_high = chi;
    return emit(j, m);
  }
  GR_HD int broadcast_heartbeat_with_hint(uint64_t clo, uint64_t chi) {  // raft.go:575-587
    need(G_CORE | G_REM);
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)S; ++j)
      if (rkind(j) == GR_SLOT_VOTER && j != self) GR_TRY(send_heartbeat(j, clo, chi));
    if (clo == 0 && chi == 0) {
#pragma unroll 1
      for (uint32_t j = 0; j < (uint32_t)S; ++j)
        if (rkind(j) == GR_SLOT_OBSERVER) {
          GR_COVER(HEARTBEAT_OBSERVER);
          GR_TRY(send_heartbeat(j, 0, 0));
        }
    }
    return 0;
  }
  GR_HD int broadcast_heartbeat() {  // raft.go:566-573
    need(G_RI);
    uint64_t clo = 0, chi = 0;
    if (ric > 0) {
      clo = sel(rilo, ric - 1);
      chi = sel(rihi, ric - 1);
    }
    return broadcast_heartbeat_with_hint(clo, chi);
  }
  GR_HD int send_timeout_now(uint64_t target) {  // raft.go:589-594
    const uint32_t j = find_slot(target);
    if (j == GR_SLOT_NONE) return GR_ESC_NONMEMBER;
    GR_COVER(TIMEOUT_NOW_SENT);
    OutMsg m;
    m.type = GR_TIMEOUT_NOW;
    return emit(j, m);
  }
  GR_HD bool leader_transfering() {  // raft.go:246-248
    need(G_CORE | G_LTT);
    return ltt != 0 && state == GR_LEADER;
  }

  // ---------------------------------------------------------------- ReadIndex (kernel step 3)
  GR_HD int ri_add(uint64_t index, uint64_t clo, uint64_t chi, uint32_t from) {  // readindex.go:43-67
    need(G_RI);
    bool dup = false;
#pragma unroll
    for (int q = 0; q < GR_Q; ++q) dup = dup || ((uint32_t)q < ric && rilo[q] == clo && rihi[q] == chi);
    if (dup) {
      GR_COVER(RI_DUP);
      return 0;
    }
    if (ric > 0 && index < sel(rii, ric - 1)) return GR_ESC_PANIC;
    if (ric >= GR_Q) return GR_ESC_CAPACITY;
    GR_COVER(RI_ADD);
#pragma unroll
    for (int q = 0; q < GR_Q; ++q) {
      const bool hit = (uint32_t)q == ric;
      rii[q] = hit ? index : rii[q];
      rilo[q] = hit ? clo : rilo[q];
      rihi[q] = hit ? chi : rihi[q];
    }
    rifrom = (rifrom & ~(0xFFu << (8 * ric))) | ((from & 0xFFu) << (8 * ric));
    riack &= ~(0xFFu << (8 * ric));
    ric++;
    dirty |= D_RI;
    return 0;
  }
  // readIndex.confirm + handleReadIndexLeaderConfirmation (readindex.go:77-116,
  // raft.go:1264-1284): ack bitmap OR, popcount quorum test, prefix release.
  GR_HD int ri_confirm(uint64_t clo, uint64_t chi, uint32_t from) {
    need(G_RI | G_CORE);
    int pos = -1;
#pragma unroll
    for (int q = 0; q < GR_Q; ++q)
      pos = (pos < 0 && (uint32_t)q < ric && rilo[q] == clo && rihi[q] == chi) ? q : pos;
    if (pos < 0) return 0;
    riack |= (1u << from) << (8 * pos);
    dirty |= D_RI;
    const uint32_t ack = (riack >> (8 * pos)) & 0xFFu;
    if (popc8(ack) + 1 < quorum()) {
      GR_COVER(RI_ACK_PENDING);
      return 0;
    }
    GR_COVER(RI_CONFIRM_RELEASE);
    const uint64_t sidx = sel(rii, (uint32_t)pos);
    bool bad = false;
#pragma unroll
    for (int q = 0; q < GR_Q; ++q) bad = bad || (q <= pos && rii[q] > sidx);
    if (bad) return GR_ESC_PANIC;
#pragma unroll 1
    for (int q = 0; q <= pos; ++q) {
      const uint32_t f = (rifrom >> (8 * q)) & 0xFFu;
      if (f == GR_SLOT_NONE || f == self) {
        GR_TRY(add_ready(sidx, sel(rilo, (uint32_t)q), sel(rihi, (uint32_t)q)));
      } else {
        GR_COVER(RI_RESP_REMOTE);
        OutMsg m;
        m.type = GR_READ_INDEX_RESP;
        m.log_index = sidx;
        m.hint = clo;
        m.hint_high = chi;
        GR_TRY(emit(f, m));
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
    return 0;
  }
  // raft.handleLeaderReadIndex (raft.go:1171-1203); from = GR_SLOT_NONE for a
  // local Peer.ReadIndex (From = NoNode).
  GR_HD int leader_read_index(uint32_t from, uint64_t clo, uint64_t chi, uint64_t mcommit) {
    need(G_CORE | G_REM);
    if (quorum() != 1) {
      if (term == 0) return GR_ESC_PANIC;  // hasCommittedEntryAtCurrentTerm :1148-1157
      uint64_t t;
      GR_TRY(term_of(committed, &t));
      if (t != term) {
        GR_COVER(RI_NOT_AT_TERM);
        return 0;
      }
      GR_TRY(ri_add(committed, clo, chi, from));
      return broadcast_heartbeat_with_hint(clo, chi);
    }
    GR_COVER(RI_SINGLE_READY);
    GR_TRY(add_ready(committed, clo, chi));
    if (from != GR_SLOT_NONE && from != self && rkind(from) == GR_SLOT_OBSERVER) {
      GR_COVER(RI_SINGLE_OBSERVER_RESP);
      OutMsg m;
      m.type = GR_READ_INDEX_RESP;
      m.log_index = committed;
      m.hint = clo;
      m.hint_high = chi;
      m.commit = mcommit;
      return emit(from, m);
    }
    return 0;
  }
  // handleFollowerReadIndex / handleFollowerLeaderTransfer / handleFollowerPropose
  // (raft.go:1346-1389): re-address the message to the known leader.
  GR_HD int forward_to_leader(const OutMsg& m, bool* dropped) {
    need(G_LID);
    *dropped = false;
    if (leader_id == 0) { *dropped = true; return 0; }
    if (m.term != 0) return GR_ESC_PANIC;  // finalizeMessageTerm, raft.go:448-450
    const uint32_t j = find_slot(leader_id);
    if (j == GR_SLOT_NONE) return GR_ESC_NONMEMBER;
    return emit(j, m);
  }

  // ---------------------------------------------------------------- log matching (kernel step 2)
  GR_HD uint64_t msg_term_at(const InMsg& m, uint64_t x) const {
    const uint64_t o = x - m.log_index - 1;
    const uint32_t nr = (m.flags >> MFL_RUNS_SHIFT) & 3u;
    return (nr == 2 && o >= m.run2) ? m.rt1 : m.rt0;
  }
  // first index in [a, b] whose local term differs from t (0 = none): the
  // segment walk restates getConflictIndex/matchTerm (logentry.go:305-312,
  // 337-343) over term runs instead of entry by entry.
  GR_HD int first_mismatch(uint64_t a, uint64_t b, uint64_t t, uint64_t* ci) {
    *ci = 0;
    if (a > b) return 0;
    if (a < lo) {  // below firstIndex-1: term() is 0
      if (t != 0) { *ci = a; return 0; }
      if (b < lo) return 0;
      a = lo;
    }
    if ((nruns == 0 || a < rs[0]) && a <= hi) return GR_ESC_TERM_WINDOW;
    uint64_t found = 0;
#pragma unroll
    for (int r = 0; r < GR_K; ++r) {
      if ((uint32_t)r < nruns) {
        const uint64_t e = (r + 1 < GR_K && (uint32_t)(r + 1) < nruns) ? rs[r + 1 < GR_K ? r + 1 : r] - 1 : hi;
        const uint64_t x = umax(a, rs[r]), y = umin(b, e);
        found = (found == 0 && x <= y && rt[r] != t) ? x : found;
      }
    }
    if (found == 0 && b > hi && t != 0) found = umax(a, hi + 1);  // beyond lastIndex: term() is 0
    *ci = found;
    return 0;
  }
  // inMemory.merge (inmemory.go:157-177) when the new entries start at or below
  // lastIndex (an append at lastIndex + 1 = markerIndex + len(entries) changes
  // neither mark): replace-all at or below markerIndex, else truncate-then-append.
  GR_HD void merge_truncate(uint64_t first) {
    need(G_INMEM);
    if (first <= imk) {
      imk = first;
      isv = first - 1;
    } else {
      isv = umin(isv, first - 1);
    }
    dirty |= D_INMEM;
  }
  GR_HD int conflict_index(const InMsg& m, uint64_t* ci) {
    *ci = 0;
    if (m.n == 0) return 0;
    const uint32_t nr = (m.flags >> MFL_RUNS_SHIFT) & 3u;
    const uint64_t a = m.log_index + 1, last = m.log_index + m.n;
    if (nr == 2) {
      const uint64_t b = m.log_index + m.run2;
      GR_TRY(first_mismatch(a, b, m.rt0, ci));
      if (*ci) return 0;
      return first_mismatch(b + 1, last, m.rt1, ci);
    }
    return first_mismatch(a, last, m.rt0, ci);
  }
  // raft.handleReplicateMessage (raft.go:953-976) with entryLog.tryAppend /
  // append / inMemory.merge (logentry.go:281-303, inmemory.go:157-177).
  GR_HD int handle_replicate(const InMsg& m, uint32_t from) {
    need(G_CORE | G_WIN);
    entries_in += m.n;
    OutMsg r;
    r.type = GR_REPLICATE_RESP;
    if (m.log_index < committed) {
      GR_COVER(REP_EARLY_ACK);
      r.log_index = committed;
      return emit(from, r);
    }
    uint64_t lt;
    GR_TRY(term_of(m.log_index, &lt));
    if (lt == m.log_term) {
      uint64_t ci;
      GR_TRY(conflict_index(m, &ci));
      if (ci == 0) GR_COVER(REP_MATCH_NO_APPEND);
      else if (ci <= hi) GR_COVER(REP_TRUNCATE);
      else GR_COVER(REP_APPEND_TAIL);
      if (ci != 0) {
        if (ci <= committed) return GR_ESC_PANIC;  // logentry.go:284-287
        if (ci > hi + 1) return GR_ESC_PANIC;      // merge would hit a hole
        const uint64_t tprev = (ci - 1 == m.log_index) ? m.log_term : msg_term_at(m, ci - 1);
        if (tprev > msg_term_at(m, ci)) return GR_ESC_PANIC;  // checkEntriesToAppend
        if (ci <= hi) merge_truncate(ci);
        win_truncate(ci);
        const uint32_t nr = (m.flags >> MFL_RUNS_SHIFT) & 3u;
        if (nr == 2) {
          GR_COVER(REP_TWO_RUNS);
          const uint64_t b2 = m.log_index + 1 + m.run2;
          if (ci < b2) win_push(ci, m.rt0);
          win_push(umax(ci, b2), m.rt1);
        } else {
          win_push(ci, m.rt0);
        }
        hi = m.log_index + m.n;
        dirty |= D_HI;  // the window is dirty only if win_truncate/win_push changed it
        append_from = append_from ? umin(append_from, ci) : ci;
      }
      const uint64_t last_idx = m.log_index + m.n;
      const uint64_t c = umin(last_idx, m.commit);
      if (c > committed) {  // commitTo, logentry.go:314-323
        if (c > hi) return GR_ESC_PANIC;
        committed = c;
        dirty |= D_COMMITTED;
      }
      r.log_index = last_idx;
    } else {
      GR_COVER(REP_REJECT);
      r.flags = MFL_REJECT;
      r.log_index = m.log_index;
      r.hint = hi;
    }
    return emit(from, r);
  }

  // ---------------------------------------------------------------- leader handlers
  GR_HD int leader_replicate_resp(const InMsg& m, uint32_t j) {  // raft.go:1205-1227
    need(G_CORE | G_REM);
    set_ractive(j, 1);
    dirty |= D_REM;
    if (!(m.flags & MFL_REJECT)) {
      GR_COVER(L_REPLICATE_RESP_ACCEPT);
      const bool paused = is_paused(rstate(j));
      if (try_update(j, m.log_index)) {
        responded_to(j);
        bool c;
        GR_TRY(try_commit(&c));
        if (c) GR_TRY(broadcast_replicate());
        else if (paused) GR_TRY(send_replicate(j));
        if (leader_transfering() && remote_id(j) == ltt && hi == sel(match, j))
          GR_TRY(send_timeout_now(ltt));
      }
    } else {
      GR_COVER(L_REPLICATE_RESP_REJECT);
      if (decrease_to(j, m.log_index, m.hint)) {
        enter_retry(j);
        GR_TRY(send_replicate(j));
      }
    }
    return 0;
  }
  GR_HD int leader_heartbeat_resp(const InMsg& m, uint32_t j) {  // raft.go:1229-1240
    need(G_CORE | G_REM);
    set_ractive(j, 1);
    wait_to_retry(j);
    dirty |= D_REM;
    if (sel(match, j) < hi) GR_TRY(send_replicate(j));
    if (m.hint != 0) GR_TRY(ri_confirm(m.hint, m.hint_high, j));
    return 0;
  }
  GR_HD int leader_leader_transfer(const InMsg& m, uint32_t j) {  // raft.go:1242-1262
    need(G_CORE | G_LEAD | G_LTT | G_REM);
    const uint64_t target = m.hint;
    if (target == 0) return GR_ESC_PANIC;
    if (leader_transfering()) return 0;
    if (node_id == target) return 0;
    ltt = target;
    zero_etick();
    dirty |= D_LTT;
    if (sel(match, j) == hi) return send_timeout_now(target);
    return 0;
  }
  GR_HD int check_quorum() {  // leaderHasQuorum + handleLeaderCheckQuorum, raft.go:262-271,1117-1123
    need(G_CORE | G_REM);
    int c = 0;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      if (rkind(j) == GR_SLOT_VOTER && ((uint32_t)j == self || ractive(j))) {
        c++;
        set_ractive(j, 0);
      }
    }
    dirty |= D_REM;
    if (c < quorum()) {
      GR_COVER(TICK_STEP_DOWN);
      return become_follower(term, 0);
    }
    GR_COVER(TICK_CHECK_QUORUM_OK);
    return 0;
  }

  // ---------------------------------------------------------------- ticks (kernel step 4)
  GR_HD int handle_election() {  // handleNodeElection, raft.go:1073-1086
    need(G_CORE | G_LEAD);
    if (state == GR_LEADER) return 0;
    if (committed > applied) {  // hasConfigChangeToApply :1055-1061
      GR_COVER(TICK_ELECTION_SKIPPED);
      return 0;
    }
    return GR_ESC_ELECTION;
  }
  GR_HD int tick() {  // raft.go:377-429
    need(G_CORE | G_TICK);
    if (state == GR_LEADER) {
      GR_COVER(TICK_LEADER);
      etick++;
      dirty |= D_ETICK;
      const bool abort = leader_transfering() && etick >= etimeout;
      if (etick >= etimeout) {
        etick = 0;
        if (flags & GR_F_CHECK_QUORUM) GR_TRY(check_quorum());
      }
      if (abort) {
        GR_COVER(TICK_TRANSFER_ABORT);
        ltt = 0;
        dirty |= D_LTT;
      }
      htick++;
      dirty |= D_HTICK;
      if (htick >= htimeout) {
        htick = 0;
        if (state == GR_LEADER) {  // only the leader has a handler
          GR_COVER(TICK_HEARTBEAT);
          GR_TRY(broadcast_heartbeat());
        }
      }
      return 0;
    }
    etick++;
    dirty |= D_ETICK;
    if (state == GR_OBSERVER) {
      GR_COVER(TICK_OBSERVER);
      return 0;
    }
    GR_COVER(TICK_FOLLOWER);
    if (etick >= retimeout && !self_removed()) {
      etick = 0;
      return handle_election();
    }
    return 0;
  }

  // ---------------------------------------------------------------- messages
  // Message k of slot j's in-mailbox mb (count byte cb): its raw words from the
  // prefetch when it holds them (pf_, k < kPfK), else from the mailbox, then one
  // decoding. A uniform mailbox's tag and term are implied by the count byte and
  // its term word (a shared pair's second message: message 0's hot fields); a
  // full record is read in one round with its hot fields: the 64-byte record as
  // four 16-byte words, decoded by type in registers (gr_layout.h Mailbox; round
  // 4 A/B against the tag first and the named fields after it: general kernel
  // 167.6 vs 173.1 us per pass on config 5).
  GR_HD void read_msg(const Mailbox& mb, uint32_t cb, uint32_t k, InMsg& m, uint32_t j = 0) const {
    const bool uni = (cb & MB_UNIFORM) != 0;
    const bool shared = k && mb_shared(cb);
    const uint32_t kh = uni && shared ? 0u : k;  // the message whose hot fields it carries
    uint64_t li;
    uint32_t cd, mt = 0;
    uint4 w0 = {0, 0, 0, 0}, w1 = w0, w2 = w0, w3 = w0;
#if defined(__HIP_DEVICE_COMPILE__)
    if (kPfWave && pf_ && k < kPfK) {
      const uint32_t lane = threadIdx.x & 63u;
      const uint8_t* ph = pf_ + (j * kPfK + kh) * kPfBytes + kPfRec + lane * 4;
      li = (uint64_t)*reinterpret_cast<const uint32_t*>(ph) | ((uint64_t)*reinterpret_cast<const uint32_t*>(ph + 256) << 32);
      cd = *reinterpret_cast<const uint32_t*>(ph + 512);
      mt = *reinterpret_cast<const uint32_t*>(ph + 768);
      if (!uni) {
        const uint8_t* pr = pf_ + (j * kPfK + k) * kPfBytes + lane * 16;
        w0 = *reinterpret_cast<const uint4*>(pr);
        w1 = *reinterpret_cast<const uint4*>(pr + 1024);
        w2 = *reinterpret_cast<const uint4*>(pr + 2048);
        w3 = *reinterpret_cast<const uint4*>(pr + 3072);
      }
    } else
#endif
    {
      li = mb.u64(kh, MF_LOG_INDEX);
      cd = mb.t32(kh, MT_CDELTA);
      if (uni) {
        mt = mb.mterm();
      } else {
        const uint4* r = reinterpret_cast<const uint4*>(mb.rec(k));
        w0 = r[0];
        w1 = r[1];
        w2 = r[2];
        w3 = r[3];
      }
    }
    if (!uni) {
      decode_record(w0, w1, w2, w3, li, cd, m);
      return;
    }
    const uint32_t tg = Mailbox::uniform_tag(cb, k);
    m.type = (uint8_t)tg;
    m.flags = (uint8_t)(tg >> 8);
    m.term = mt;
    m.n = 0; m.run2 = 0;
    m.log_index = 0; m.log_term = 0; m.commit = 0; m.hint = 0; m.hint_high = 0; m.rt0 = 0; m.rt1 = 0;
    if (m.type == GR_REPLICATE) {  // uniform Replicates are compact: LogTerm = Term, <= 1 entry at Term
      m.log_index = li;
      m.n = (m.flags & MFL_N1) ? 1u : 0u;
      m.log_term = m.term;
      m.commit = commit_of(cd, li);
      m.rt0 = m.n ? m.term : 0;
    } else {  // an accept (MB_RESP): a shared pair's second is at message 0's LogIndex + 1
      m.log_index = li + (shared ? (uint64_t)k : 0ull);
    }
  }
  // A full-record message from its cold record's words and its hot LogIndex and
  // Commit offset (gr_layout.h Mailbox).
  GR_HD static void decode_record(const uint4& w0, const uint4& w1, const uint4& w2, const uint4& w3, uint64_t li,
                                  uint32_t cd, InMsg& m) {
    {
      m.type = (uint8_t)(w0.x & 0xFFu);
      m.flags = (uint8_t)((w0.x >> 8) & 0xFFu);
      m.term = w0.y;
      m.n = 0; m.run2 = 0;
      m.log_index = 0; m.log_term = 0; m.commit = 0; m.hint = 0; m.hint_high = 0; m.rt0 = 0; m.rt1 = 0;
      const uint64_t commit = (uint64_t)w2.x | ((uint64_t)w2.y << 32), hint = (uint64_t)w2.z | ((uint64_t)w2.w << 32),
                     hint_high = (uint64_t)w3.x | ((uint64_t)w3.y << 32);
      switch (m.type) {
        case GR_REPLICATE:
          m.log_index = li;
          if (m.flags & MFL_COMPACT) {
            m.n = (m.flags & MFL_N1) ? 1u : 0u;
            m.log_term = m.term;
            m.commit = commit_of(cd, li);
            m.rt0 = m.n ? m.term : 0;
            break;
          }
          m.n = w0.z;
          m.log_term = w1.x;
          m.commit = (m.flags & MFL_WIDE_COMMIT) ? commit : commit_of(cd, li);
          if (m.n) {
            m.rt0 = w1.y;
            if (((m.flags >> MFL_RUNS_SHIFT) & 3u) == 2) {
              m.run2 = w0.w;
              m.rt1 = w1.z;
            }
          }
          break;
        case GR_REPLICATE_RESP:
          m.log_index = li;
          if (m.flags & MFL_REJECT) m.hint = hint;
          break;
        case GR_HEARTBEAT:
          m.commit = commit;
          m.hint = hint;
          m.hint_high = hint_high;
          break;
        case GR_HEARTBEAT_RESP:
          m.hint = hint;
          m.hint_high = hint_high;
          break;
        default:
          m.n = w0.z;
          m.run2 = w0.w;
          m.log_index = li;
          m.log_term = w1.x;
          m.commit = commit;
          m.hint = hint;
          m.hint_high = hint_high;
          m.rt0 = w1.y;
          m.rt1 = w1.z;
          break;
      }
    }
  }
  GR_HD OutMsg as_out(const InMsg& m) const {
    OutMsg o;
    o.type = m.type;
    o.flags = m.flags;
    o.n = m.n;
    o.run2 = m.run2;
    o.term = m.term;
    o.log_index = m.log_index;
    o.log_term = m.log_term;
    o.commit = m.commit;
    o.hint = m.hint;
    o.hint_high = m.hint_high;
    o.rt0 = m.rt0;
    o.rt1 = m.rt1;
    return o;
  }
  // raft.Handle (raft.go:1014-1053) + defaultHandle handler tables (:1481-1527)
  GR_HD int handle(const InMsg& m, uint32_t from) {
    need(G_CORE);
    const uint32_t t = m.type;
    if (m.term != 0 && m.term != term) {  // onMessageTermNotMatched
      if (m.term > term) {
        if (t == GR_REQUEST_VOTE) return GR_ESC_UNSUPPORTED;  // dropRequestVoteFromHighTermNode + vote
        const uint64_t lid = is_leader_message(t) ? remote_id(from) : 0;
        if (state == GR_OBSERVER) {
          GR_COVER(TERM_HIGHER_OBSERVER);
          GR_TRY(become_observer(m.term, lid));
        } else {
          GR_COVER(TERM_HIGHER);
          GR_TRY(become_follower(m.term, lid));
        }
      } else {
        if (is_leader_message(t) && (flags & GR_F_CHECK_QUORUM)) {
          GR_COVER(TERM_LOWER_NOOP);
          OutMsg o;
          o.type = GR_NOOP;
          return emit(from, o);
        }
        GR_COVER(TERM_LOWER_DROP);
        return 0;
      }
    }
    if (state == GR_LEADER) {
      switch (t) {
        case GR_REPLICATE_RESP:
        case GR_HEARTBEAT_RESP:
        case GR_SNAPSHOT_STATUS:
        case GR_UNREACHABLE:
        case GR_LEADER_TRANSFER: {
          need(G_REM);
          if (rkind(from) == GR_SLOT_EMPTY) {  // lw: no remote (raft.go:1466-1479)
            GR_COVER(L_RESP_NONMEMBER);
            return 0;
          }
          if (t == GR_REPLICATE_RESP) return leader_replicate_resp(m, from);
          if (t == GR_HEARTBEAT_RESP) {
            GR_COVER(L_HEARTBEAT_RESP);
            return leader_heartbeat_resp(m, from);
          }
          if (t == GR_LEADER_TRANSFER) {
            GR_COVER(L_LEADER_TRANSFER);
            return leader_leader_transfer(m, from);
          }
          if (t == GR_UNREACHABLE) {
            GR_COVER(L_UNREACHABLE);
            enter_retry(from);
            dirty |= D_REM;
            return 0;
          }
          GR_COVER(L_SNAPSHOT_STATUS);
          if (rstate(from) != GR_SNAPSHOT_ST) return 0;  // SnapshotStatus :1286-1299
          need(G_SNAP);
          if (m.flags & MFL_REJECT) {
            put(snap, from, (uint64_t)0);
            dirty |= D_SNAP;
          }
          become_retry(from);  // becomeWait = becomeRetry + retryToWait
          set_rstate(from, GR_WAIT);
          dirty |= D_REM;
          return 0;
        }
        case GR_READ_INDEX: GR_COVER(L_READ_INDEX_MSG); return leader_read_index(from, m.hint, m.hint_high, m.commit);
        case GR_LEADER_HEARTBEAT: GR_COVER(L_LEADER_HEARTBEAT); return broadcast_heartbeat();
        case GR_CHECK_QUORUM: GR_COVER(L_CHECK_QUORUM_MSG); return check_quorum();
        case GR_ELECTION: GR_COVER(L_ELECTION); return 0;
        case GR_PROPOSE: GR_COVER(L_PROPOSE_FWD); return leader_forwarded_propose(m);
        case GR_REQUEST_VOTE: return GR_ESC_UNSUPPORTED;
        default: GR_COVER(L_NIL); return 0;  // nil handler
      }
    }
    if (state == GR_FOLLOWER || state == GR_OBSERVER) {
      const bool obs = state == GR_OBSERVER;
      switch (t) {
        case GR_REPLICATE:  // raft.go:1359-1363
          if (obs) GR_COVER(O_REPLICATE);
          else GR_COVER(F_REPLICATE);
          zero_etick();
          set_leader_from(from);
          return handle_replicate(m, from);
        case GR_HEARTBEAT: {  // raft.go:1365-1369, 923-931
          if (obs) GR_COVER(O_HEARTBEAT);
          else GR_COVER(F_HEARTBEAT);
          zero_etick();
          set_leader_from(from);
          if (m.commit > committed) {
            if (m.commit > hi) return GR_ESC_PANIC;
            committed = m.commit;
            dirty |= D_COMMITTED;
          }
          OutMsg o;
          o.type = GR_HEARTBEAT_RESP;
          o.hint = m.hint;
          o.hint_high = m.hint_high;
          return emit(from, o);
        }
        case GR_READ_INDEX_RESP:  // raft.go:1391-1399
          if (obs) GR_COVER(O_READ_INDEX_RESP);
          else GR_COVER(F_READ_INDEX_RESP);
          zero_etick();
          set_leader_from(from);
          return add_ready(m.log_index, m.hint, m.hint_high);
        case GR_READ_INDEX: {
          if (obs) GR_COVER(O_READ_INDEX_FWD);
          else GR_COVER(F_READ_INDEX_FWD);
          bool d;
          return forward_to_leader(as_out(m), &d);
        }
        case GR_LEADER_TRANSFER: {
          if (obs) { GR_COVER(O_DROPPED); return 0; }
          GR_COVER(F_LEADER_TRANSFER_FWD);
          bool d;
          return forward_to_leader(as_out(m), &d);
        }
        case GR_ELECTION:
          if (obs) { GR_COVER(O_DROPPED); return 0; }
          GR_COVER(F_ELECTION);
          return handle_election();
        case GR_PROPOSE: {  // handleFollowerPropose / handleObserverPropose (raft.go:1346-1357, 1322)
          if (obs) GR_COVER(O_PROPOSE_FWD);
          else GR_COVER(F_PROPOSE_FWD);
          bool d;
          return forward_to_leader(as_out(m), &d);
        }
        case GR_INSTALL_SNAPSHOT: return GR_ESC_UNSUPPORTED;
        case GR_REQUEST_VOTE:
        case GR_TIMEOUT_NOW:
          if (obs) { GR_COVER(O_DROPPED); return 0; }
          return GR_ESC_UNSUPPORTED;
        default: GR_COVER(F_NIL); return 0;
      }
    }
    switch (t) {  // candidate: every non-nil handler changes role or votes
      case GR_PROPOSE: GR_COVER(C_PROPOSE); return 0;  // handleCandidatePropose only logs
      case GR_HEARTBEAT:
      case GR_REPLICATE:
      case GR_INSTALL_SNAPSHOT:
      case GR_REQUEST_VOTE_RESP:
      case GR_ELECTION:
      case GR_REQUEST_VOTE: return GR_ESC_UNSUPPORTED;
      default: GR_COVER(C_NIL); return 0;
    }
  }

  // appendEntries + broadcastReplicateMessage (raft.go:643-654, 1144-1145)
  GR_HD int append_proposal(uint32_t n) {
    need(G_WIN | G_REM);
    if (nruns > 0 && last_run_term() > term) return GR_ESC_PANIC;  // checkEntriesToAppend
    const uint64_t first = hi + 1;
    win_push(first, term);
    hi += n;
    dirty |= D_HI | D_REM;
    try_update(self, hi);
    if (quorum() == 1) {
      bool c;
      GR_TRY(try_commit(&c));
    }
    GR_TRY(broadcast_replicate());
    if (!propose_first) propose_first = first;
    return 0;
  }
  // handleLeaderPropose (raft.go:1125-1146) for a batch a follower forwarded
  // (handleFollowerPropose :1346-1357). The device takes only appends, so the
  // host can attribute the entries (gr_peer_result.propose_first): a drop
  // (selfRemoved, leader transfer) or a config change goes to the host.
  GR_HD int leader_forwarded_propose(const InMsg& m) {
    if (m.flags & MFL_REJECT) return GR_ESC_CONFIG_CHANGE;
    if (m.n == 0 || self_removed() || leader_transfering()) return GR_ESC_UNSUPPORTED;
    GR_TRY(append_proposal(m.n));
    fwd_n++;
    fwd_entries += m.n;
    return 0;
  }

  // raft.handleLeaderPropose + appendEntries (raft.go:1125-1146, 643-654), or
  // the follower/observer forward and the candidate drop.
  GR_HD int propose(uint32_t n, bool has_cc) {
    need(G_CORE);
    if (state == GR_LEADER) {
      if (self_removed()) { GR_COVER(PROP_DROP_SELF_REMOVED); prop_result = GR_PROP_DROPPED; return 0; }
      if (leader_transfering()) { GR_COVER(PROP_DROP_TRANSFER); prop_result = GR_PROP_DROPPED; return 0; }
      if (has_cc) return GR_ESC_CONFIG_CHANGE;
      GR_COVER(PROP_APPEND);
      GR_TRY(append_proposal(n));
      prop_result = GR_PROP_APPENDED;
      return 0;
    }
    if (state == GR_CANDIDATE) {
      GR_COVER(PROP_CANDIDATE);
      prop_result = GR_PROP_DROPPED;
      return 0;
    }
    OutMsg o;
    o.type = GR_PROPOSE;
    o.n = n;  // one run of n entries at term 0: appendEntries has not stamped them (raft.go:643-650)
    o.flags = (uint8_t)((1u << MFL_RUNS_SHIFT) | (has_cc ? MFL_REJECT : 0u));  // reject bit: holds a ConfigChangeEntry
    bool dropped;
    GR_TRY(forward_to_leader(o, &dropped));
    if (dropped) GR_COVER(PROP_DROP_NO_LEADER);
    else GR_COVER(PROP_FORWARD);
    prop_result = dropped ? GR_PROP_DROPPED : GR_PROP_FORWARDED;
    return 0;
  }

  // ---------------------------------------------------------------- driver
  GR_HD void begin() {
    outu = 0;
    loaded = 0;
    dirty = 0;
    snapz = 0;
    rtrc = 0;
    prop_result = 0;
    rand_used = false;
    append_from = 0;
    propose_first = 0;
    fwd_n = 0;
    fwd_entries = 0;
    msgs_in = 0;
    msgs_out = 0;
    entries_in = 0;
    outcnt = 0;
  }
  // Process items [0, limit); returns an escalation code and the item index
  // where it stopped (*at), or 0 with *at = number of items processed.
  GR_HD int run(uint32_t limit, uint32_t* at) {
    uint32_t item = 0;
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)S; ++j) {
      const uint32_t g = in_gpos(j);
      if (g == NOPOS) continue;
      const Mailbox mb = kp.in.at(g);
      const uint32_t cb = GR_LANE_PRELOAD ? sel(pcb_, j) : (uint32_t)mb.cnt(), c = mb_n(cb);
#pragma unroll 1
      for (uint32_t k = 0; k < c; ++k) {
        if (item == limit) { *at = item; return 0; }
        if (k == kp.in.depth) { *at = item; return GR_ESC_CAPACITY; }  // overflowed mailbox
        // its cold fields did not fit the exchange's side buffer (gr_io.h side_pack)
        if (!(cb & MB_UNIFORM) && (cb & MB_COLD_LOST)) { *at = item; return GR_ESC_CAPACITY; }
        InMsg m;
        read_msg(mb, cb, k, m, j);
        if (m.type == MT_WIDE) { *at = item; return GR_ESC_WIDE_TERM; }  // terms >= 2^32: host path
        const int e = handle(m, j);
        if (e) { *at = item; return e; }
        msgs_in++;
        item++;
      }
    }
    if (kp.has_locals) {
      const uint32_t lf = GR_LANE_PRELOAD ? plf_ : kp.ln.u8(LR_LFLAGS)[i];
      const uint32_t nt = GR_LANE_PRELOAD ? pnt_ : kp.ln.u32(LR_TICKS)[i];
      const uint32_t nq = GR_LANE_PRELOAD ? pnq_ : kp.ln.u32(LR_QTICKS)[i];
      const uint32_t np = GR_LANE_PRELOAD ? pnp_ : kp.ln.u32(LR_PROPOSE)[i];
      if (lf & LF_READ_INDEX) {
        if (item == limit) { *at = item; return 0; }
        need(G_CORE);
        const uint64_t clo = kp.ln.u64(LR_RI_LO)[i], chi = kp.ln.u64(LR_RI_HI)[i];
        int e = 0;
        if (state == GR_LEADER) {
          e = leader_read_index(GR_SLOT_NONE, clo, chi, 0);
        } else if (state != GR_CANDIDATE) {
          GR_COVER(RI_LOCAL_FORWARD);
          OutMsg o;
          o.type = GR_READ_INDEX;
          o.hint = clo;
          o.hint_high = chi;
          bool d;
          e = forward_to_leader(o, &d);
        }
        if (e) { *at = item; return e; }
        item++;
      }
#pragma unroll 1
      for (uint32_t t = 0; t < nt; ++t) {
        if (item == limit) { *at = item; return 0; }
        const int e = tick();
        if (e) { *at = item; return e; }
        item++;
      }
      if (nq) {  // quiescedTick x nq: electionTick++ only (raft.go:431-433); one item
        if (item == limit) { *at = item; return 0; }
        GR_COVER(QTICK);
        need(G_ETICK);
        etick += nq;
        dirty |= D_ETICK;
        item++;
      }
      if (np) {
        if (item == limit) { *at = item; return 0; }
        const int e = propose(np, (lf & LF_PROPOSE_CC) != 0);
        if (e) { *at = item; return e; }
        item++;
      }
    }
    *at = item;
    return 0;
  }

  // Kernel body for one lane: run, and on escalation re-run the prefix on the
  // pristine state so the escalating item is left entirely to the host.
  GR_HD bool step(LaneStats* ls) {
    GR_COVER(GENERAL_LANE);
    uint32_t at = 0, limit = 0xFFFFFFFFu;
    int esc = 0;
    preload();
    prefetch();
#pragma unroll 1
    for (int attempt = 0; attempt < 2; ++attempt) {  // one call site keeps run() inlined
      begin();
      // the groups nearly every handed-over lane reads, in one round of loads
      // instead of one dependent round per group as the handlers reach them
      need(G_CORE | G_WIN | G_REM | G_ETICK | G_LID);
      if (attempt == 0) tclk[0] = lane_clock(kp);
      const int e = run(limit, &at);
      if (attempt == 0) tclk[1] = lane_clock(kp);
      if (!e) break;
      esc = e;  // second attempt re-runs the prefix and cannot escalate
      limit = at;
    }
    store();
    tclk[2] = lane_clock(kp);
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)S; ++j) {  // every routed mailbox is rewritten each pass
      const uint32_t g = out_gpos(j);
      if (g == NOPOS) continue;
      const uint32_t c = (outcnt >> (3 * j)) & 7u, u = (uint32_t)(outu >> (5 * j)) & 31u;
      kp.out.at(g).cnt() = (uint8_t)(c && !(u & 1u) ? c | MB_UNIFORM | ((u & 2u) ? (uint32_t)MB_RESP : 0u) |
                                                         ((u >> 2) << MB_N1_SHIFT)
                                                   : c);
    }
    uint8_t rf = 0;
    if (esc) {
      GR_COVER_ESC(esc);
      rf |= RF_ESCALATED;
      kp.ln.u8(LR_ESC_REASON)[i] = (uint8_t)esc;
      kp.ln.u32(LR_ESC_ITEM)[i] = at;
    }
    if (prop_result) {  // propose_first = last_index - n + 1 (gr_layout.h)
      rf |= RF_PROPOSE;
      kp.ln.u8(LR_PROP_RESULT)[i] = (uint8_t)prop_result;
    }
    if (rtrc) {
      rf |= RF_READY;
      kp.ln.u8(LR_RTR_COUNT)[i] = (uint8_t)rtrc;
    }
    if (append_from) {
      rf |= RF_APPEND;
      kp.ln.u64(LR_APPEND_FROM)[i] = append_from;
    }
    if (fwd_n) {
      rf |= RF_FORWARDED;
      kp.ln.u8(LR_FWD_COUNT)[i] = (uint8_t)fwd_n;
      kp.ln.u32(LR_FWD_ENTRIES)[i] = fwd_entries;
    }
    if (dirty & (D_TERM | D_VOTE)) rf |= RF_HARDSTATE;
    kp.ln.u8(LR_RFLAGS)[i] = rf;
    const bool adv = (dirty & D_COMMITTED) && committed > committed0;
    const bool lead = state == GR_LEADER;
    ls->leader_commit = adv && lead;
    ls->follower_commit = adv && !lead;
    ls->escalated = esc != 0;
    ls->msgs_in = msgs_in;
    ls->msgs_out = msgs_out;
    ls->leader_in = lead ? msgs_in : 0;
    ls->leader_out = lead ? msgs_out : 0;
    ls->entries = entries_in;
    return true;
  }
};

}  // namespace gr
