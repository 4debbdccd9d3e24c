// gr_host.h — helpers shared by libgpuraft.so and the test-only CPU harness:
// gr_peer <-> SoA row conversion and the message codec of the mailbox spaces
// (gr_layout.h). No HIP runtime calls. The codec, validation and result
// derivation are __host__ __device__: the boundary kernels (gr_io.h) run the
// same functions on the device.
#pragma once
#include <algorithm>
#include <cstring>
#include <vector>

#include "gr_layout.h"

namespace gr {
namespace host {

// Row accessors between gr_peer and the SoA state rows (also run by the
// load/sync passes of gr_io.h on the device).
// The header word of a record (gr_layout.h): small fields plus the device bits.
__host__ __device__ inline uint64_t header_of(const gr_peer& g, uint32_t S) {
  uint32_t sl = 0;
  for (uint32_t j = 0; j < S && j < 7 && g.leader_id; ++j)
    if (!sl && g.remote_id[j] == g.leader_id) sl = j + 1;
  const uint32_t flags = (g.flags & F_PUBLIC) | (g.leader_transfer_target ? F_LTT : 0u) |
                         (g.election_tick == 0 ? F_ETZ : 0u) | (sl << F_LSLOT_SHIFT);
  const uint32_t n = g.n_runs <= GR_K ? g.n_runs : GR_K;
  const bool gelo = n && g.run_start[n - 1] >= g.first_index_m1;
  uint64_t rb = 0;
  for (uint32_t j = 0; j < S; ++j)
    rb |= (uint64_t)((g.remotes[j].state & 3u) | ((g.remotes[j].active & 1u) << 2) | ((g.remotes[j].kind & 3u) << 3))
          << (5 * j);
  uint64_t h = h_make(g.state, g.self_slot, n, gelo, flags, g.read_index_count, rb);
  if (has_run_bits((int)S) && n) h |= run_bits(n, g.run_start[n - 1], g.run_term[n - 1], g.term, g.committed);
  // a leader's sync bits where the record's rows already hold the values they
  // imply (gr_layout.h): a loaded steady leader starts as FastLane leaves one
  // (the rows are written too, so the bits only let the lanes skip them)
  if (has_sync_bits((int)S) && g.state == GR_LEADER) {
    for (uint32_t j = 0; j < S; ++j) {
      if (g.remotes[j].next == g.last_index + 1) h |= 1ull << (H_NX_SHIFT + j);
      if (j != g.self_slot && g.last_index >= 2 && g.remotes[j].match == g.last_index - 2)
        h |= 1ull << (H_MP_SHIFT + j);
    }
    if (g.self_slot < S && g.remotes[g.self_slot].match == g.last_index) h |= 1ull << H_MS_BIT;
  }
  return h;
}
__host__ __device__ inline void set_header(gr_peer& g, uint32_t S, uint64_t h) {
  g.state = (uint8_t)h_state(h);
  g.self_slot = (uint8_t)h_self(h);
  g.n_runs = (uint8_t)h_nruns(h);
  g.flags = (uint8_t)(h_flags(h) & F_PUBLIC);
  g.read_index_count = (uint8_t)h_ric(h);
  const uint64_t rb = h_rb(h);
  for (uint32_t j = 0; j < S; ++j) {
    g.remotes[j].state = (uint8_t)rb_state(rb, j);
    g.remotes[j].active = (uint8_t)rb_active(rb, j);
    g.remotes[j].kind = (uint8_t)rb_kind(rb, j);
  }
}

// The header's sync bits (gr_layout.h): the rows they cover are stale and the
// values follow from lastIndex. Applied after every row of g has been set.
__host__ __device__ inline void resolve_sync(gr_peer& g, uint32_t S, uint64_t h) {
  if (!has_sync_bits((int)S)) return;  // wider groups: those header bits are remote state
  for (uint32_t j = 0; j < S; ++j) {
    if (h_nx(h, j)) g.remotes[j].next = g.last_index + 1;
    if (h_mp(h, j) && j != g.self_slot) g.remotes[j].match = g.last_index - 2;
  }
  if (h_ms(h) && g.self_slot < S) g.remotes[g.self_slot].match = g.last_index;
}

// Rows are converted in ascending order: SR_HDR (which carries n_runs) comes
// before the right-aligned run rows that need it.
__host__ __device__ inline uint64_t get_u64_row(const gr_peer& g, uint32_t row, uint32_t S) {
  if (row < SR_HDR) {
    // marker_index == 0: a freshly loaded group (newEntryLog, logentry.go:86-95)
    const bool fresh = g.marker_index == 0;
    const uint64_t v[] = {g.term, g.vote, g.committed, g.applied, g.last_index, g.first_index_m1,
                          g.leader_id, g.leader_transfer_target, g.node_id, g.election_tick,
                          g.heartbeat_tick, g.randomized_election_timeout, g.election_timeout,
                          g.heartbeat_timeout, g.entry_size_ub,
                          fresh ? g.last_index : g.saved_to, fresh ? g.last_index + 1 : g.marker_index,
                          fresh ? g.first_index_m1 : g.log_applied};
    return v[row];
  }
  if (row == SR_HDR) return header_of(g, S);
  const uint32_t n = g.n_runs <= GR_K ? g.n_runs : GR_K;
  if (row < SR_RUN_TERM) {
    const int k = (int)(row - SR_RUN_START) - (int)(GR_K - n);
    return k >= 0 ? g.run_start[k] : 0;
  }
  if (row < SR_REMOTE) {
    const int k = (int)(row - SR_RUN_TERM) - (int)(GR_K - n);
    return k >= 0 ? g.run_term[k] : 0;
  }
  uint32_t r = row - SR_REMOTE;
  if (r < S) return g.remotes[r].match;
  r -= S;
  if (r < S) return g.remotes[r].next;
  r -= S;
  if (r < S) return g.remotes[r].snapshot_index;
  r -= S;
  if (r < S) return g.remote_id[r];
  r -= S;
  if (r < GR_Q) return g.read_index[r].index;
  r -= GR_Q;
  if (r < GR_Q) return g.read_index[r].ctx_low;
  r -= GR_Q;
  return g.read_index[r].ctx_high;
}
__host__ __device__ inline void set_u64_row(gr_peer& g, uint32_t row, uint32_t S, uint64_t v) {
  if (row < SR_HDR) {
    uint64_t* f[] = {&g.term, &g.vote, &g.committed, &g.applied, &g.last_index, &g.first_index_m1,
                     &g.leader_id, &g.leader_transfer_target, &g.node_id, &g.election_tick,
                     &g.heartbeat_tick, &g.randomized_election_timeout, &g.election_timeout,
                     &g.heartbeat_timeout, &g.entry_size_ub, &g.saved_to, &g.marker_index, &g.log_applied};
    *f[row] = v;
    return;
  }
  if (row == SR_HDR) { set_header(g, S, v); return; }
  const uint32_t n = g.n_runs <= GR_K ? g.n_runs : GR_K;  // set by the SR_HDR row before
  if (row < SR_RUN_TERM) {
    const int k = (int)(row - SR_RUN_START) - (int)(GR_K - n);
    if (k >= 0) g.run_start[k] = v;
    return;
  }
  if (row < SR_REMOTE) {
    const int k = (int)(row - SR_RUN_TERM) - (int)(GR_K - n);
    if (k >= 0) g.run_term[k] = v;
    return;
  }
  uint32_t r = row - SR_REMOTE;
  if (r < S) { g.remotes[r].match = v; return; }
  r -= S;
  if (r < S) { g.remotes[r].next = v; return; }
  r -= S;
  if (r < S) { g.remotes[r].snapshot_index = v; return; }
  r -= S;
  if (r < S) { g.remote_id[r] = v; return; }
  r -= S;
  if (r < GR_Q) { g.read_index[r].index = v; return; }
  r -= GR_Q;
  if (r < GR_Q) { g.read_index[r].ctx_low = v; return; }
  r -= GR_Q;
  g.read_index[r].ctx_high = v;
}
// u8 rows: rifrom[Q], riack[Q]
__host__ __device__ inline uint8_t get_u8_row(const gr_peer& g, uint32_t row, uint32_t) {
  if (row < GR_Q) return g.read_index[row].from_slot;
  return g.read_index[row - GR_Q].ack_bits;
}
__host__ __device__ inline void set_u8_row(gr_peer& g, uint32_t row, uint32_t, uint8_t v) {
  if (row < GR_Q) g.read_index[row].from_slot = v;
  else g.read_index[row - GR_Q].ack_bits = v;
}

__host__ __device__ inline int validate_msg(const gr_message& m, uint32_t S, uint32_t cap) {
  if (m.peer >= cap || m.slot >= S) return GR_EINVAL;
  if (m.type > GR_TIMEOUT_NOW) return GR_EINVAL;
  if (m.n_runs > 2) return GR_EINVAL;
  if (m.n_entries == 0 && m.n_runs != 0) return GR_EINVAL;
  if (m.n_entries != 0 && m.n_runs == 0) return GR_EINVAL;
  if (m.n_runs == 2 && (m.run2_offset == 0 || m.run2_offset >= m.n_entries)) return GR_EINVAL;
  return GR_OK;
}

__host__ __device__ inline void encode_msg(const Mailbox& mb, uint32_t k, const gr_message& m) {
  if (wide_term(m.term, m.log_term, m.run_term[0], m.run_term[1])) {  // cannot travel: receiver escalates
    mb.type(k) = MT_WIDE;
    return;
  }
  mb.type(k) = m.type;
  uint8_t fl = (uint8_t)((m.reject ? MFL_REJECT : 0) | (m.n_runs << MFL_RUNS_SHIFT));
  if (m.type == GR_REPLICATE) {
    uint32_t cd;
    if (commit_delta(m.commit, m.log_index, &cd)) mb.t32(k, MT_CDELTA) = cd;
    else fl |= MFL_WIDE_COMMIT;
  }
  mb.flags(k) = fl;
  mb.n(k) = m.n_entries;
  mb.run2(k) = m.run2_offset;
  mb.t32(k, MT_TERM) = (uint32_t)(m.term);
  mb.u64(k, MF_LOG_INDEX) = m.log_index;
  mb.t32(k, MT_LOG_TERM) = (uint32_t)(m.log_term);
  mb.u64(k, MF_COMMIT) = m.commit;
  mb.u64(k, MF_HINT) = m.hint;
  mb.u64(k, MF_HINT_HIGH) = m.hint_high;
  mb.t32(k, MT_RT0) = (uint32_t)(m.run_term[0]);
  mb.t32(k, MT_RT1) = (uint32_t)(m.run_term[1]);
}

// Can m travel in a uniform mailbox (gr_layout.h MB_UNIFORM)? 0 = no; else
// 1 | 2 for a ReplicateResp accept | 4 for a Replicate carrying its one entry.
// A uniform Replicate is compact (LogTerm = Term, at most one entry at Term,
// narrow Commit), so its compact decode equals the full one.
__host__ __device__ inline uint32_t uniform_class(const gr_message& m) {
  if (wide_term(m.term, m.log_term, m.run_term[0], m.run_term[1])) return 0;
  if (m.type == GR_REPLICATE_RESP) return m.reject ? 0u : 3u;  // an accept carries Term and LogIndex
  if (m.type != GR_REPLICATE) return 0;
  uint32_t cd;
  if (!commit_delta(m.commit, m.log_index, &cd) || m.log_term != m.term) return 0;
  if (m.n_entries == 0) return m.n_runs == 0 ? 1u : 0u;
  return (m.n_entries == 1 && m.n_runs == 1 && m.run_term[0] == m.term) ? 5u : 0u;
}
// The count byte of a mailbox whose `count` messages (at(q), q < count) are
// encoded: MB_UNIFORM with the term word written when they all allow it.
template <class MsgAt>
__host__ __device__ inline uint8_t count_byte(const Mailbox& mb, uint32_t count, MsgAt at) {
  if (count == 0 || count > kUniformMax) return (uint8_t)count;
  uint32_t cb = count | MB_UNIFORM;
  uint64_t t0 = 0;
  for (uint32_t q = 0; q < count; ++q) {
    const gr_message m = at(q);
    const uint32_t u = uniform_class(m);
    if (!u) return (uint8_t)count;
    if (q == 0) {
      t0 = m.term;
      if (u & 2) cb |= MB_RESP;
    } else if (m.term != t0 || ((u & 2) != 0) != ((cb & MB_RESP) != 0)) {
      return (uint8_t)count;
    }
    if (u & 4) cb |= 1u << (MB_N1_SHIFT + q);
  }
  mb.mterm() = (uint32_t)t0;
  return (uint8_t)cb;
}

// Decode one message; fields a type does not carry on the device are zero.
__host__ __device__ inline gr_message decode_msg(const Mailbox& mb, uint32_t k) {
  gr_message m{};  // no padding in gr_message: every byte is a zeroed field
  const uint32_t cb = mb.cnt(), tg = mb.tag_at(k, cb);  // MB_UNIFORM: tag and term implied
  m.type = (uint8_t)tg;
  const uint8_t fl = (uint8_t)(tg >> 8);
  m.reject = (fl & MFL_REJECT) ? 1 : 0;
  m.n_runs = (fl >> MFL_RUNS_SHIFT) & 3u;
  m.term = (uint64_t)mb.term_at(k, cb);
  switch (m.type) {
    case GR_REPLICATE:
      if (fl & MFL_COMPACT) {  // gr_layout.h: LogTerm = Term, <= 1 entry at Term, narrow Commit
        m.log_index = mb.log_index_at(k, cb);  // a shared mailbox: message 0's
        m.n_entries = (fl & MFL_N1) ? 1u : 0u;
        m.n_runs = m.n_entries ? 1u : 0u;
        m.log_term = m.term;
        m.commit = commit_of(mb.cdelta_at(k, cb), m.log_index);
        if (m.n_entries) m.run_term[0] = m.term;
        break;
      }
      m.n_entries = mb.n(k);
      m.log_index = mb.u64(k, MF_LOG_INDEX);
      m.log_term = (uint64_t)mb.t32(k, MT_LOG_TERM);
      m.commit = (fl & MFL_WIDE_COMMIT) ? mb.u64(k, MF_COMMIT) : commit_of(mb.t32(k, MT_CDELTA), m.log_index);
      if (m.n_entries) m.run_term[0] = (uint64_t)mb.t32(k, MT_RT0);
      if (m.n_runs == 2) {
        m.run2_offset = mb.run2(k);
        m.run_term[1] = (uint64_t)mb.t32(k, MT_RT1);
      }
      break;
    case GR_REPLICATE_RESP:  // the device writes Hint only on a reject
      m.log_index = mb.log_index_at(k, cb);  // a shared mailbox: message 0's + k
      if (m.reject) m.hint = mb.u64(k, MF_HINT);
      break;
    case GR_HEARTBEAT:
      m.commit = mb.u64(k, MF_COMMIT);
      m.hint = mb.u64(k, MF_HINT);
      m.hint_high = mb.u64(k, MF_HINT_HIGH);
      break;
    case GR_HEARTBEAT_RESP:
      m.hint = mb.u64(k, MF_HINT);
      m.hint_high = mb.u64(k, MF_HINT_HIGH);
      break;
    default:
      m.n_entries = mb.n(k);
      m.run2_offset = mb.run2(k);
      m.log_index = mb.u64(k, MF_LOG_INDEX);
      m.log_term = (uint64_t)mb.t32(k, MT_LOG_TERM);
      m.commit = mb.u64(k, MF_COMMIT);
      m.hint = mb.u64(k, MF_HINT);
      m.hint_high = mb.u64(k, MF_HINT_HIGH);
      m.run_term[0] = (uint64_t)mb.t32(k, MT_RT0);
      m.run_term[1] = (uint64_t)mb.t32(k, MT_RT1);
      break;
  }
  return m;
}



// Pack a gr_step inbox: lanes = sorted unique peers with input; in-space
// mailboxes only for (lane, slot) pairs that carry messages, filled in
// arrival order; out-space identity lane*S + slot. Returns GR_* status.
struct PackedInbox {
  std::vector<uint32_t> peers;    // lane -> peer
  std::vector<uint32_t> in_pos;   // [S][nl]
  std::vector<uint32_t> out_pos;  // [S][nl]
  std::vector<gr_local_input> locals;  // by lane
  uint32_t in_positions = 1, out_positions = 0;
  std::vector<std::pair<uint32_t, uint32_t>> msg_pos;  // message k -> (position, k-th in mailbox)
  uint32_t lane(uint32_t pp) const {
    return (uint32_t)(std::lower_bound(peers.begin(), peers.end(), pp) - peers.begin());
  }
};

inline int pack_inbox(const gr_inbox* in, uint32_t S, uint32_t max_peers, PackedInbox* pk) {
  pk->peers.clear();
  for (size_t k = 0; k < in->n_msgs; ++k) {
    const int r = validate_msg(in->msgs[k], S, max_peers);
    if (r) return r;
    pk->peers.push_back(in->msgs[k].peer);
  }
  for (size_t k = 0; k < in->n_locals; ++k) {
    if (in->locals[k].peer >= max_peers) return GR_EINVAL;
    pk->peers.push_back(in->locals[k].peer);
  }
  std::sort(pk->peers.begin(), pk->peers.end());
  pk->peers.erase(std::unique(pk->peers.begin(), pk->peers.end()), pk->peers.end());
  const uint32_t nl = (uint32_t)pk->peers.size();
  std::vector<uint32_t> mcount((size_t)nl * S, 0);
  for (size_t k = 0; k < in->n_msgs; ++k) {
    // more than GR_C messages in one mailbox: the first GR_C travel, the
    // mailbox is marked overflowed and the receiver escalates there (CAPACITY)
    ++mcount[(size_t)pk->lane(in->msgs[k].peer) * S + in->msgs[k].slot];
  }
  // slot-major positions: consecutive lanes use consecutive mailboxes of
  // every field array (coalesced on the device)
  pk->in_pos.assign((size_t)S * nl, NOPOS);
  uint32_t npos = 0;
  for (uint32_t j = 0; j < S; ++j)
    for (uint32_t l = 0; l < nl; ++l)
      if (mcount[(size_t)l * S + j]) pk->in_pos[(size_t)j * nl + l] = npos++;
  pk->in_positions = std::max<uint32_t>(npos, 1);
  pk->out_positions = std::max<uint32_t>(nl * S, 1);
  pk->out_pos.resize((size_t)S * nl);
  for (uint32_t j = 0; j < S; ++j)
    for (uint32_t l = 0; l < nl; ++l) pk->out_pos[(size_t)j * nl + l] = j * nl + l;
  std::vector<uint32_t> fill((size_t)nl * S, 0);
  pk->msg_pos.resize(in->n_msgs);
  for (size_t k = 0; k < in->n_msgs; ++k) {
    const gr_message& m = in->msgs[k];
    const uint32_t l = pk->lane(m.peer);
    pk->msg_pos[k] = {pk->in_pos[(size_t)m.slot * nl + l], fill[(size_t)l * S + m.slot]++};
  }
  pk->locals.assign(nl, gr_local_input{});
  for (size_t k = 0; k < in->n_locals; ++k) pk->locals[pk->lane(in->locals[k].peer)] = in->locals[k];
  return GR_OK;
}

// First index of inMemory.entriesToSave() (inmemory.go:101-108), 0 when it is
// empty: idx = savedTo + 1; "nothing to save" when idx - markerIndex (uint64,
// wrapping) exceeds len(entries) = lastIndex + 1 - markerIndex.
__host__ __device__ inline uint64_t save_from(uint64_t saved_to, uint64_t marker, uint64_t last_index) {
  const uint64_t idx = saved_to + 1;
  if (idx - marker > last_index + 1 - marker) return 0;
  return idx <= last_index ? idx : 0;
}

// The proposal fields of a result record from the lane rows (gr_layout.h RF_*):
// propose_first is not stored, it follows from last_index since proposals are
// the only appends of a pass that reports them.
__host__ __device__ inline void derive_proposals(gr_peer_result* pr, uint8_t rf, uint8_t pres, uint64_t last_index,
                             uint32_t local_n, uint8_t fwd_n, uint32_t fwd_entries) {
  uint64_t n = 0;
  if (rf & RF_PROPOSE) {
    pr->propose_result = pres;
    if (pres == GR_PROP_APPENDED) n += local_n;
  }
  if (rf & RF_FORWARDED) {
    pr->n_forwarded = fwd_n;
    pr->forwarded_entries = fwd_entries;
    n += fwd_entries;
  }
  if (n) pr->propose_first = last_index - n + 1;
}

// The result record of lane l (stepping peer p) from the lane and state rows
// after a pass: RF_* flags (gr_layout.h) select the per-pass fields; the
// pb.Update fields (committed, last_index, save_from, term, vote) come from state.
__host__ __device__ inline gr_peer_result make_result(const LaneBase& L, const StateBase& st, uint32_t l, uint32_t p) {
  gr_peer_result pr{};
  pr.peer = p;
  const uint8_t rf = L.u8(LR_RFLAGS)[l];
  if (rf & RF_ESCALATED) {
    pr.escalation = L.u8(LR_ESC_REASON)[l];
    pr.esc_item = L.u32(LR_ESC_ITEM)[l];
  }
  pr.last_index = st.u64(SR_LAST_INDEX)[p];
  if (rf & (RF_PROPOSE | RF_FORWARDED))
    derive_proposals(&pr, rf, L.u8(LR_PROP_RESULT)[l], pr.last_index, L.u32(LR_PROPOSE)[l], L.u8(LR_FWD_COUNT)[l],
                     L.u32(LR_FWD_ENTRIES)[l]);
  if (rf & RF_APPEND) pr.append_from = L.u64(LR_APPEND_FROM)[l];
  if (rf & RF_READY) {
    pr.n_ready = L.u8(LR_RTR_COUNT)[l];
    for (int q = 0; q < GR_Q; ++q) {
      if (q < pr.n_ready) {
        pr.ready[q].index = L.u64(LR_RTR_INDEX + q)[l];
        pr.ready[q].ctx_low = L.u64(LR_RTR_LO + q)[l];
        pr.ready[q].ctx_high = L.u64(LR_RTR_HI + q)[l];
      }
    }
  }
  pr.committed = st.u64(SR_COMMITTED)[p];
  pr.save_from = save_from(st.u64(SR_SAVED_TO)[p], st.u64(SR_MARKER)[p], pr.last_index);
  pr.term = st.u64(SR_TERM)[p];
  pr.vote = st.u64(SR_VOTE)[p];
  return pr;
}

// entryLog.commitUpdate (logentry.go:325-335) on the state rows of peer p:
// inMemory.savedLogTo(stable_log_to, stable_log_term), then entryLog.applied =
// applied_to and inMemory.appliedLogTo (inmemory.go:92-139). Returns 0 (rows
// written), 1 where the reference panics (invalid applyto) or 2 when the term
// of stable_log_to lies below the term-run window; nothing is written then.
__host__ __device__ inline int32_t commit_marks(const StateBase& st, uint32_t p, const gr_update_commit& u) {
  uint64_t mk = st.u64(SR_MARKER)[p], sv = st.u64(SR_SAVED_TO)[p], ap = st.u64(SR_LOG_APPLIED)[p];
  const uint64_t last = st.u64(SR_LAST_INDEX)[p], committed = st.u64(SR_COMMITTED)[p];
  const bool inmem = last + 1 > mk;  // len(entries) > 0
  if (u.stable_log_to > 0) {
    const uint64_t i = u.stable_log_to;
    if (inmem && i >= mk && i <= last) {
      const uint64_t h = st.u64(SR_HDR)[p];
      uint32_t nr = h_nruns(h);
      if (nr > GR_K) nr = GR_K;
      uint64_t t = 0;
      bool known = false;
      for (uint32_t r = 0; r < nr; ++r) {  // last run starting at or below i
        if (st.u64(SR_RUN_START + run_row(nr, r))[p] <= i) {
          t = st.u64(SR_RUN_TERM + run_row(nr, r))[p];
          known = true;
        }
      }
      if (!known) return 2;
      if (t == u.stable_log_term) sv = i;
    }
  }
  if (u.applied_to > 0) {
    const uint64_t a = u.applied_to;
    if (a < ap || a > committed) return 1;  // "invalid applyto" panic
    ap = a;
    if (inmem && a >= mk && a <= last) mk = a;
  }
  st.u64(SR_MARKER)[p] = mk;
  st.u64(SR_SAVED_TO)[p] = sv;
  st.u64(SR_LOG_APPLIED)[p] = ap;
  return 0;
}

// ---- compact boundary records (gpuraft.h gr_cmsg / gr_clocal / gr_cresult)
// Compact form of a message, or false when it needs an ext record. The
// compact record always carries peer, type and slot (the sort keys).
__host__ __device__ inline bool cmsg_of(const gr_message& m, gr_cmsg* c) {
  c->peer = m.peer;
  c->type = m.type;
  c->slot = m.slot;
  c->flags = 0;
  c->pad = 0;
  c->term = (uint32_t)m.term;
  c->aux = 0;
  c->log_index = m.log_index;
  if ((m.term >> 32) || m.hint_high || m.run2_offset || m.run_term[1] || m.reject > 1) return false;
  uint8_t fl = m.reject ? GR_CM_REJECT : 0;
  if (m.n_entries) {
    if (m.n_entries != 1 || m.n_runs != 1 || m.run_term[0] != m.term) return false;
    fl |= GR_CM_ENTRY;
  } else if (m.n_runs || m.run_term[0]) {
    return false;
  }
  if (m.log_term) {
    if (m.log_term != m.term) return false;
    fl |= GR_CM_LOG_TERM;
  }
  if (m.commit && m.hint) return false;
  uint32_t d = 0;
  if (m.commit) {
    if (!commit_delta(m.commit, m.log_index, &d)) return false;
    fl |= GR_CM_COMMIT;
  }
  if (m.hint) {
    if (!commit_delta(m.hint, m.log_index, &d)) return false;
    fl |= GR_CM_HINT;
  }
  c->aux = d;
  c->flags = fl;
  return true;
}
// Messages a compact record stands for: two for a GR_CM_PAIR record.
__host__ __device__ inline uint32_t cmsg_n(const gr_cmsg& c) {
  return (c.flags & (GR_CM_PAIR | GR_CM_EXT)) == GR_CM_PAIR ? 2u : 1u;
}
// Message k (0, or 1 of a pair) of a compact record (not GR_CM_EXT) in full.
__host__ __device__ inline gr_message msg_of(const gr_cmsg& c, uint32_t k = 0) {
  gr_message m{};
  m.peer = c.peer;
  m.type = c.type;
  m.slot = c.slot;
  m.reject = (c.flags & GR_CM_REJECT) ? 1 : 0;
  m.term = c.term;
  // a pair's second accept acknowledges one index more; its second Replicate
  // repeats LogIndex (gpuraft.h GR_CM_PAIR)
  m.log_index = c.log_index + (k && c.type == GR_REPLICATE_RESP ? 1u : 0u);
  if (c.flags & GR_CM_LOG_TERM) m.log_term = m.term;
  if (c.flags & GR_CM_COMMIT) m.commit = commit_of(c.aux, c.log_index);
  if (c.flags & GR_CM_HINT) m.hint = commit_of(c.aux, c.log_index);
  if (c.flags & (k ? GR_CM_ENTRY2 : GR_CM_ENTRY)) {
    m.n_entries = 1;
    m.n_runs = 1;
    m.run_term[0] = m.term;
  }
  return m;
}
// The pair record of two consecutive compact records of one mailbox, or false
// when GR_CM_PAIR cannot carry them (gpuraft.h).
__host__ __device__ inline bool pair_of(const gr_cmsg& a, const gr_cmsg& b, gr_cmsg* out) {
  if (((a.flags | b.flags) & (GR_CM_EXT | GR_CM_PAIR | GR_CM_ENTRY2)) || a.peer != b.peer || a.slot != b.slot ||
      a.type != b.type || a.term != b.term || a.aux != b.aux)
    return false;
  if (a.type == GR_REPLICATE) {
    if (b.log_index != a.log_index || (a.flags & ~GR_CM_ENTRY) != (b.flags & ~GR_CM_ENTRY)) return false;
  } else if (a.type == GR_REPLICATE_RESP) {
    if ((a.flags & GR_CM_REJECT) || a.flags != b.flags || b.log_index != a.log_index + 1) return false;
  } else {
    return false;
  }
  *out = a;
  out->flags = (uint8_t)(a.flags | GR_CM_PAIR | ((b.flags & GR_CM_ENTRY) ? GR_CM_ENTRY2 : 0));
  return true;
}
__host__ __device__ inline int validate_cmsg(const gr_cmsg& c, const gr_message* ext, uint32_t n_ext, uint32_t S,
                                             uint32_t cap) {
  if (c.peer >= cap || c.slot >= S || c.type > GR_TIMEOUT_NOW) return GR_EINVAL;
  if (c.flags & GR_CM_EXT) {
    if (c.aux >= n_ext) return GR_EINVAL;
    const gr_message& m = ext[c.aux];
    if (m.peer != c.peer || m.slot != c.slot || m.type != c.type) return GR_EINVAL;
    return validate_msg(m, S, cap);
  }
  if ((c.flags & GR_CM_ENTRY2) && !(c.flags & GR_CM_PAIR)) return GR_EINVAL;
  if ((c.flags & GR_CM_PAIR) && !(c.type == GR_REPLICATE ||
                                  (c.type == GR_REPLICATE_RESP && !(c.flags & (GR_CM_REJECT | GR_CM_ENTRY2)))))
    return GR_EINVAL;
  if ((c.flags & GR_CM_COMMIT) && (c.flags & GR_CM_HINT)) return GR_EINVAL;
  return GR_OK;
}
__host__ __device__ inline gr_message expand_cmsg(const gr_cmsg& c, const gr_message* ext, uint32_t k = 0) {
  return (c.flags & GR_CM_EXT) ? ext[c.aux] : msg_of(c, k);
}
__host__ __device__ inline bool clocal_of(const gr_local_input& x, gr_clocal* c) {
  c->peer = x.peer;
  c->propose_entries = x.propose_entries;
  c->ticks = (uint16_t)x.ticks;
  c->quiesced_ticks = (uint8_t)x.quiesced_ticks;
  c->flags = x.propose_has_config_change ? GR_CL_CONFIG_CHANGE : 0;
  c->ext = 0;
  c->rand = x.rand;
  return !(x.read_index || x.read_ctx_low || x.read_ctx_high || x.ticks > 0xFFFFu || x.quiesced_ticks > 0xFFu ||
           x.propose_has_config_change > 1);
}
__host__ __device__ inline gr_local_input expand_clocal(const gr_clocal& c, const gr_local_input* ext) {
  if (c.flags & GR_CL_EXT) return ext[c.ext];
  gr_local_input x{};
  x.peer = c.peer;
  x.propose_entries = c.propose_entries;
  x.ticks = c.ticks;
  x.quiesced_ticks = c.quiesced_ticks;
  x.propose_has_config_change = (c.flags & GR_CL_CONFIG_CHANGE) ? 1 : 0;
  x.rand = c.rand;
  return x;
}
__host__ __device__ inline bool validate_clocal(const gr_clocal& c, const gr_local_input* ext, uint32_t n_ext,
                                                uint32_t cap) {
  if (c.peer >= cap || (c.flags & ~(GR_CL_EXT | GR_CL_CONFIG_CHANGE))) return false;
  return !(c.flags & GR_CL_EXT) || (c.ext < n_ext && ext[c.ext].peer == c.peer);
}
// A lane's result needs the full record (ReadyToRead, forwarded batches, State change).
__host__ __device__ inline bool result_needs_ext(uint8_t rf) {
  return (rf & (RF_READY | RF_FORWARDED | RF_HARDSTATE)) != 0;
}
// The compact result (gpuraft.h gr_cresult); false when it needs the full
// record (an escalation, or an index range the relative fields cannot carry).
__host__ __device__ inline bool cresult_of(const gr_peer_result& r, gr_cresult* c) {
  *c = gr_cresult{};
  c->peer = r.peer;
  c->escalation = r.escalation;
  c->propose_result = r.propose_result;
  c->aux = r.esc_item;
  c->last_index = r.last_index;
  const uint64_t lag = r.last_index - r.committed, save = r.save_from ? r.last_index - r.save_from + 1 : 0;
  c->commit_lag = (uint32_t)lag;
  c->save_count = (uint8_t)save;
  return !r.escalation && r.committed <= r.last_index && !(lag >> 32) && r.save_from <= r.last_index + 1 &&
         save <= 0xFFu;
}

inline uint64_t space_total_bytes(uint32_t n_chunks, uint32_t positions, uint32_t depth = GR_C) {
  return (uint64_t)n_chunks * space_chunk_bytes_pc(space_pad_positions(positions), depth);
}

inline SpaceView make_view(const void* base, uint32_t n_chunks, uint32_t positions, uint32_t depth = GR_C) {
  SpaceView v;
  v.base = (uint8_t*)base;
  v.n_chunks = n_chunks;
  v.pc = space_pad_positions(positions);
  v.hot_bytes = space_hot_chunk_bytes_pc(v.pc, depth);
  v.cold_bytes = space_cold_chunk_bytes_pc(v.pc, depth);
  v.depth = depth;
  return v;
}

inline void encode_inbox(const gr_inbox* in, const PackedInbox& pk, void* space) {
  const SpaceView v = make_view(space, 1, pk.in_positions);
  std::vector<std::vector<size_t>> by_pos(pk.in_positions);  // messages of each mailbox, in order
  for (size_t k = 0; k < in->n_msgs; ++k) {
    const Mailbox mb = v.at(pk.msg_pos[k].first);
    if (pk.msg_pos[k].second >= GR_C) {
      mb.cnt() = (uint8_t)(GR_C + 1);  // overflow marker
      continue;
    }
    encode_msg(mb, pk.msg_pos[k].second, in->msgs[k]);
    mb.cnt() = (uint8_t)(pk.msg_pos[k].second + 1);
    by_pos[pk.msg_pos[k].first].push_back(k);
  }
  for (uint32_t g = 0; g < pk.in_positions; ++g) {
    const Mailbox mb = v.at(g);
    if (by_pos[g].empty() || mb.cnt() > GR_C) continue;
    mb.cnt() = count_byte(mb, (uint32_t)by_pos[g].size(), [&](uint32_t q) { return in->msgs[by_pos[g][q]]; });
  }
}

inline void decode_outbox(const void* space, const PackedInbox& pk, uint32_t S, std::vector<gr_message>* out) {
  const SpaceView v = make_view(space, 1, pk.out_positions);
  const uint32_t nl = (uint32_t)pk.peers.size();
  for (uint32_t l = 0; l < nl; ++l) {
    for (uint32_t j = 0; j < S; ++j) {
      const Mailbox mb = v.at(j * nl + l);
      const uint32_t c = std::min<uint32_t>(mb_n(mb.cnt()), GR_C);
      for (uint32_t k = 0; k < c; ++k) {
        gr_message m = decode_msg(mb, k);
        m.peer = pk.peers[l];
        m.slot = (uint8_t)j;
        out->push_back(m);
      }
    }
  }
}

// Route tables of a replica-major population (lane i = r*G + g) whose every
// entry is base[dir][r][j] + g (or NOPOS for the whole (r, j) block) become
// RT_AFFINE: the kernel computes positions instead of reading 8*S bytes of
// tables per lane. Tries each replica count R <= S that divides n.
inline bool detect_affine_routes(const uint32_t* in_pos, const uint32_t* out_pos, uint32_t n, uint32_t S,
                                 uint32_t* base /* [2][GR_SMAX][GR_SMAX] */, uint32_t* g_out, uint32_t* r_out) {
  if (n == 0) return false;
  for (uint32_t R = 1; R <= S && R <= GR_SMAX; ++R) {
    if (n % R) continue;
    const uint32_t G = n / R;
    bool ok = true;
    for (uint32_t d = 0; d < 2 && ok; ++d) {
      const uint32_t* t = d ? out_pos : in_pos;
      for (uint32_t r = 0; r < R && ok; ++r) {
        for (uint32_t j = 0; j < S && ok; ++j) {
          const uint32_t* row = t + (size_t)j * n + (size_t)r * G;
          const uint32_t b = row[0];
          if (b != NOPOS && (uint64_t)b + G - 1 >= NOPOS) { ok = false; break; }
          for (uint32_t x = 0; x < G; ++x) {
            const uint32_t want = b == NOPOS ? NOPOS : b + x;
            if (row[x] != want) { ok = false; break; }
          }
          base[(d * GR_SMAX + r) * GR_SMAX + j] = b;
        }
      }
    }
    if (ok) {
      *g_out = G;
      *r_out = R;
      return true;
    }
  }
  return false;
}

// An affine route table that is exactly the replica-major loopback (RT_LOOPBACK).
inline bool is_loopback(const uint32_t* base, uint32_t G, uint32_t R, uint32_t S) {
  const uint64_t n = (uint64_t)R * G;
  for (uint32_t r = 0; r < R; ++r)
    for (uint32_t j = 0; j < S; ++j) {
      const bool none = j == r || j >= R;
      const uint64_t bi = none ? NOPOS : j * n + (uint64_t)r * G;
      const uint64_t bo = none ? NOPOS : r * n + (uint64_t)j * G;
      if (base[(0 * GR_SMAX + r) * GR_SMAX + j] != bi || base[(1 * GR_SMAX + r) * GR_SMAX + j] != bo)
        return false;
    }
  return true;
}

// Local-input rows of a lane block (host copies).
__host__ __device__ inline void locals_to_rows(const gr_local_input& x, uint32_t* ticks, uint32_t* qticks, uint32_t* prop,
                           uint8_t* lflags, uint64_t* rlo, uint64_t* rhi, uint64_t* rnd, uint32_t* lword) {
  *ticks = x.ticks;
  *qticks = x.quiesced_ticks;
  *prop = x.propose_entries;
  *lflags = (uint8_t)((x.read_index ? LF_READ_INDEX : 0) | (x.propose_has_config_change ? LF_PROPOSE_CC : 0));
  *rlo = x.read_ctx_low;
  *rhi = x.read_ctx_high;
  *rnd = x.rand;
  *lword = local_word(*ticks, *qticks, *prop, *lflags);
}

}  // namespace host
}  // namespace gr
