// gr_io.h — the boundary's data movement on the device (gr_step, gr_collect_results).
//
// gr_step takes caller-owned gr_message / gr_local_input records and returns
// gr_message / gr_peer_result records (include/gpuraft.h). Packing those on
// the host (sort the peers, assign mailboxes, SoA-encode, then decode every
// mailbox back) cost 1.75 s per pass at 1M groups x 3, four orders of
// magnitude above the step kernels. Here the records cross PCIe as they are
// and every transformation is a data-parallel pass in HBM:
//
//   inbox:  mark_inputs (validate, flag peers with input)
//           -> exclusive scan of the flags: lane_of_peer, nl (lanes = peers
//              with input, ascending, as node.go's step worker visits them)
//           -> lane_peers (peer_of_lane into LR_LANE_PEER)
//           -> msg_keys + stable counting sort by mailbox (slot-major position
//              j*nl + lane; key_count, scan, key_scatter, key_order): arrival
//              order inside a mailbox survives
//           -> encode_sorted (SoA mailbox fields, the count byte; more than
//              GR_C messages mark the mailbox overflowed, as the host packer did)
//           -> local_winner + fill_locals (one gr_local_input per lane, the
//              last one given wins, zero rows for lanes without one)
//   outbox: out_counts -> exclusive scan -> pack_outbox (lane, slot, arrival order)
//           pack_results (one gr_peer_result per lane)
//
// Routes are RT_IDENTITY both ways (mailbox j*nl + lane), so no route table is
// built or read. The codec functions are the same ones the test-only host
// packer uses (gr_host.h), so the records are bit-identical.
#pragma once
#include "gpuraft_wire.h"
#include "gr_host.h"
#include "gr_scan.h"

namespace gr {
namespace io {

constexpr int kIoBlock = 256;

__device__ inline uint32_t io_tid() { return blockIdx.x * kIoBlock + threadIdx.x; }
__device__ inline uint32_t io_stride() { return gridDim.x * kIoBlock; }

// Validate every record (gr_host.h validate_msg) and flag the peers with input.
__global__ void mark_inputs(const gr_message* msgs, uint32_t n_msgs, const gr_local_input* loc, uint32_t n_loc,
                            uint32_t S, uint32_t cap, uint32_t* mark, uint32_t* err) {
  for (uint32_t k = io_tid(); k < n_msgs + n_loc; k += io_stride()) {
    if (k < n_msgs) {
      const gr_message& m = msgs[k];
      if (host::validate_msg(m, S, cap) != GR_OK) {
        atomicOr(err, 1u);
        continue;
      }
      mark[m.peer] = 1;
    } else {
      const uint32_t p = loc[k - n_msgs].peer;
      if (p >= cap) {
        atomicOr(err, 1u);
        continue;
      }
      mark[p] = 1;
    }
  }
}

// nl = last exclusive-scan value + last flag; err copied beside it (one D2H).
__global__ void finish_lanes(const uint32_t* mark, const uint32_t* lane_of_peer, uint32_t cap, const uint32_t* err,
                             uint32_t* out2) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out2[0] = cap ? lane_of_peer[cap - 1] + mark[cap - 1] : 0;
    out2[1] = *err;
  }
}

__global__ void lane_peers(const uint32_t* mark, const uint32_t* lane_of_peer, uint32_t cap, uint32_t* peer_of_lane) {
  for (uint32_t p = io_tid(); p < cap; p += io_stride())
    if (mark[p]) peer_of_lane[lane_of_peer[p]] = p;
}

__global__ void msg_keys(const gr_message* msgs, uint32_t n, const uint32_t* lane_of_peer, uint32_t nl,
                         uint32_t* keys, uint32_t* idx) {
  for (uint32_t k = io_tid(); k < n; k += io_stride()) {
    keys[k] = (uint32_t)msgs[k].slot * nl + lane_of_peer[msgs[k].peer];
    idx[k] = k;
  }
}

// ---- the stable sort of the inbox's mailbox keys (bounded: key < positions),
// hand-written as a counting sort: count the records of every mailbox (each
// record takes a slot of its mailbox), scan the counts, scatter, then restore
// arrival order inside each mailbox (record index ascending; mailboxes hold a
// few records, more than GR_C overflow and escalate anyway).
__global__ void key_count(const uint32_t* keys, uint32_t n, uint32_t* cnt, uint32_t* slot) {
  for (uint32_t k = io_tid(); k < n; k += io_stride()) slot[k] = atomicAdd(cnt + keys[k], 1u);
}
__global__ void key_scatter(const uint32_t* keys, const uint32_t* slot, uint32_t n, const uint32_t* base,
                            uint32_t* skeys, uint32_t* sidx) {
  for (uint32_t k = io_tid(); k < n; k += io_stride()) {
    const uint32_t key = keys[k], at = base[key] + slot[k];
    skeys[at] = key;
    sidx[at] = k;  // msg_keys' idx[k] = k
  }
}
// Arrival order inside mailbox `key`: its record indexes ascending (insertion
// sort for the few records a mailbox holds). Only the first GR_C + 1 records in
// arrival order matter beyond that (encode_sorted writes GR_C of them and marks
// the mailbox overflowed; the receiver escalates CAPACITY at message GR_C), so an
// overfull mailbox (malformed or adversarial input) gets a partial selection of
// its GR_C + 1 smallest indexes: O(c * (GR_C + 1)) on its thread, not a full sort.
__global__ void key_order(const uint32_t* cnt, const uint32_t* base, uint32_t nkeys, uint32_t* sidx) {
  for (uint32_t key = io_tid(); key < nkeys; key += io_stride()) {
    const uint32_t c = cnt[key];
    if (c < 2) continue;
    uint32_t* a = sidx + base[key];
    if (c <= 16) {
      for (uint32_t i = 1; i < c; ++i) {
        const uint32_t x = a[i];
        uint32_t j = i;
        while (j > 0 && a[j - 1] > x) {
          a[j] = a[j - 1];
          --j;
        }
        a[j] = x;
      }
      continue;
    }
    for (uint32_t t = 0; t <= (uint32_t)GR_C; ++t) {
      uint32_t m = t;
      for (uint32_t u = t + 1; u < c; ++u) m = a[u] < a[m] ? u : m;
      const uint32_t x = a[t];
      a[t] = a[m];
      a[m] = x;
    }
  }
}

// Sorted record s is the r-th of its mailbox, r = run of equal keys before it
// (looked at up to GR_C back: a mailbox holds GR_C). The last record of a run
// writes the count byte (GR_C + 1 = overflowed; the receiver escalates CAPACITY
// at the first message that did not travel).
__global__ void encode_sorted(const gr_message* msgs, const uint32_t* skeys, const uint32_t* sidx, uint32_t n,
                              SpaceView v) {
  for (uint32_t s = io_tid(); s < n; s += io_stride()) {
    const uint32_t key = skeys[s];
    uint32_t r = 0;
    while (r <= (uint32_t)GR_C && r < s && skeys[s - r - 1] == key) ++r;
    const Mailbox mb = v.at(key);
    if (r < (uint32_t)GR_C) host::encode_msg(mb, r, msgs[sidx[s]]);
    if (s + 1 == n || skeys[s + 1] != key)  // the mailbox's last record: its count byte (uniform when it can be)
      mb.cnt() = r < (uint32_t)GR_C ? host::count_byte(mb, r + 1, [&](uint32_t q) { return msgs[sidx[s - r + q]]; })
                                    : (uint8_t)(GR_C + 1);
  }
}

// The last record given for a peer wins (win[lane] = 1 + its index).
// lane_of_peer == nullptr: lane = peer (gr_set_locals).
__global__ void local_winner(const gr_local_input* loc, uint32_t n, const uint32_t* lane_of_peer, uint32_t* win) {
  for (uint32_t k = io_tid(); k < n; k += io_stride()) {
    const uint32_t p = loc[k].peer;
    atomicMax(win + (lane_of_peer ? lane_of_peer[p] : p), k + 1);
  }
}

__global__ void fill_locals(const gr_local_input* loc, const uint32_t* win, uint32_t nl, LaneBase L) {
  for (uint32_t l = io_tid(); l < nl; l += io_stride()) {
    gr_local_input x{};
    if (win[l]) x = loc[win[l] - 1];
    host::locals_to_rows(x, L.u32(LR_TICKS) + l, L.u32(LR_QTICKS) + l, L.u32(LR_PROPOSE) + l, L.u8(LR_LFLAGS) + l,
                         L.u64(LR_RI_LO) + l, L.u64(LR_RI_HI) + l, L.u64(LR_RAND) + l, L.u32(LR_LWORD) + l);
  }
}

// Messages each lane emitted (RT_IDENTITY out space, mailbox j*nl + lane).
__global__ void out_counts(SpaceView out, uint32_t nl, uint32_t S, uint32_t* oc) {
  for (uint32_t l = io_tid(); l < nl; l += io_stride()) {
    uint32_t c = 0;
    for (uint32_t j = 0; j < S; ++j) {
      const uint32_t x = mb_n(out.at(j * nl + l).cnt());
      c += x < (uint32_t)GR_C ? x : (uint32_t)GR_C;
    }
    oc[l] = c;
  }
}

__global__ void finish_total(const uint32_t* oc, const uint32_t* off, uint32_t nl, uint32_t* total) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *total = nl ? off[nl - 1] + oc[nl - 1] : 0;
}

__global__ void pack_outbox(SpaceView out, uint32_t nl, uint32_t S, const uint32_t* off,
                            const uint32_t* peer_of_lane, gr_message* rec) {
  for (uint32_t l = io_tid(); l < nl; l += io_stride()) {
    uint32_t o = off[l];
    const uint32_t peer = peer_of_lane[l];
    for (uint32_t j = 0; j < S; ++j) {
      const Mailbox mb = out.at(j * nl + l);
      const uint32_t x = mb_n(mb.cnt());
      const uint32_t c = x < (uint32_t)GR_C ? x : (uint32_t)GR_C;
      for (uint32_t k = 0; k < c; ++k) {
        gr_message m = host::decode_msg(mb, k);
        m.peer = peer;
        m.slot = (uint8_t)j;
        rec[o++] = m;
      }
    }
  }
}

// Result records of lanes [first, first + n) (RF_* flags, gr_layout.h).
// peer_of_lane == nullptr: lane l steps peer l.
__global__ void pack_results(LaneBase L, StateBase st, const uint32_t* peer_of_lane, uint32_t first, uint32_t n,
                             gr_peer_result* out) {
  for (uint32_t x = io_tid(); x < n; x += io_stride())
    out[x] = host::make_result(L, st, first + x, peer_of_lane ? peer_of_lane[x] : first + x);
}

// ---- compact records (gr_step_compact): the same passes over gr_cmsg /
// gr_clocal, with ext records for what does not fit (gr_host.h codec).
struct CInbox {
  const gr_cmsg* msgs;
  const gr_message* ext;
  const gr_clocal* loc;
  const gr_local_input* lext;
  uint32_t n_msgs, n_ext, n_loc, n_lext;
};

__global__ void mark_inputs_c(CInbox in, uint32_t S, uint32_t cap, uint32_t* mark, uint32_t* err) {
  for (uint32_t k = io_tid(); k < in.n_msgs + in.n_loc; k += io_stride()) {
    if (k < in.n_msgs) {
      const gr_cmsg c = in.msgs[k];
      if (host::validate_cmsg(c, in.ext, in.n_ext, S, cap) != GR_OK) {
        atomicOr(err, 1u);
        continue;
      }
      mark[c.peer] = 1;
    } else {
      const gr_clocal c = in.loc[k - in.n_msgs];
      if (!host::validate_clocal(c, in.lext, in.n_lext, cap)) {
        atomicOr(err, 1u);
        continue;
      }
      mark[c.peer] = 1;
    }
  }
}

__global__ void msg_keys_c(const gr_cmsg* msgs, uint32_t n, const uint32_t* lane_of_peer, uint32_t nl, uint32_t* keys,
                           uint32_t* idx) {
  for (uint32_t k = io_tid(); k < n; k += io_stride()) {
    keys[k] = (uint32_t)msgs[k].slot * nl + lane_of_peer[msgs[k].peer];
    idx[k] = k;
  }
}

// encode_sorted over compact records (expanded in registers). A GR_CM_PAIR
// record is two messages: a record's first message lands after the messages of
// the mailbox's earlier records.
__global__ void encode_sorted_c(CInbox in, const uint32_t* skeys, const uint32_t* sidx, SpaceView v) {
  const uint32_t n = in.n_msgs;
  for (uint32_t s = io_tid(); s < n; s += io_stride()) {
    const uint32_t key = skeys[s];
    uint32_t nrec = 0, r = 0;  // earlier records of the mailbox, their messages (counted up to overflow)
    while (r <= (uint32_t)GR_C && nrec < s && skeys[s - nrec - 1] == key) {
      r += host::cmsg_n(in.msgs[sidx[s - nrec - 1]]);
      ++nrec;
    }
    const Mailbox mb = v.at(key);
    const gr_cmsg c = in.msgs[sidx[s]];
    const uint32_t nm = host::cmsg_n(c);
    for (uint32_t q = 0; q < nm; ++q)
      if (r + q < (uint32_t)GR_C) host::encode_msg(mb, r + q, host::expand_cmsg(c, in.ext, q));
    if (s + 1 == n || skeys[s + 1] != key)
      mb.cnt() = r + nm <= (uint32_t)GR_C ? host::count_byte(mb, r + nm, [&](uint32_t q) {
        uint32_t x = s - nrec;  // the mailbox's first record
        for (;;) {
          const gr_cmsg& cx = in.msgs[sidx[x]];
          const uint32_t k = host::cmsg_n(cx);
          if (q < k) return host::expand_cmsg(cx, in.ext, q);
          q -= k;
          ++x;
        }
      }) : (uint8_t)(GR_C + 1);
  }
}

__global__ void local_winner_c(const gr_clocal* loc, uint32_t n, const uint32_t* lane_of_peer, uint32_t* win) {
  for (uint32_t k = io_tid(); k < n; k += io_stride()) atomicMax(win + lane_of_peer[loc[k].peer], k + 1);
}

__global__ void fill_locals_c(CInbox in, const uint32_t* win, uint32_t nl, LaneBase L) {
  for (uint32_t l = io_tid(); l < nl; l += io_stride()) {
    gr_local_input x{};
    if (win[l]) x = host::expand_clocal(in.loc[win[l] - 1], in.lext);
    host::locals_to_rows(x, L.u32(LR_TICKS) + l, L.u32(LR_QTICKS) + l, L.u32(LR_PROPOSE) + l, L.u8(LR_LFLAGS) + l,
                         L.u64(LR_RI_LO) + l, L.u64(LR_RI_HI) + l, L.u64(LR_RAND) + l, L.u32(LR_LWORD) + l);
  }
}

// The compact records of one out mailbox, in order (a pair of messages that
// GR_CM_PAIR carries is one record; a message that fits no compact form is an
// ext record): rec(compact record, full message or nullptr).
template <class Rec>
__device__ inline void mailbox_records(const Mailbox& mb, uint32_t peer, uint32_t slot, Rec rec) {
  const uint32_t x = mb_n(mb.cnt());
  const uint32_t c = x < (uint32_t)GR_C ? x : (uint32_t)GR_C;
  for (uint32_t k = 0; k < c;) {
    gr_message m = host::decode_msg(mb, k);
    m.peer = peer;
    m.slot = (uint8_t)slot;
    gr_cmsg cm;
    const bool fits = host::cmsg_of(m, &cm);
    if (fits && k + 1 < c) {
      gr_message m2 = host::decode_msg(mb, k + 1);
      m2.peer = peer;
      m2.slot = (uint8_t)slot;
      gr_cmsg c2, pr;
      if (host::cmsg_of(m2, &c2) && host::pair_of(cm, c2, &pr)) {
        rec(pr, (const gr_message*)nullptr);
        k += 2;
        continue;
      }
    }
    rec(cm, fits ? (const gr_message*)nullptr : &m);
    ++k;
  }
}

// Per lane: records (high word) and those needing an ext record (low word) in
// one u64, so one scan gives both output offsets; rx = 1 when the result needs
// the full record.
__global__ void out_counts_c(SpaceView out, LaneBase L, StateBase st, uint32_t nl, uint32_t S, uint64_t* oc,
                             uint32_t* rx) {
  for (uint32_t l = io_tid(); l < nl; l += io_stride()) {
    uint32_t c = 0, e = 0;
    for (uint32_t j = 0; j < S; ++j)
      mailbox_records(out.at(j * nl + l), 0u, j, [&](const gr_cmsg&, const gr_message* full) {
        ++c;
        e += full ? 1u : 0u;
      });
    oc[l] = ((uint64_t)c << 32) | e;
    gr_cresult cr;
    rx[l] = host::result_needs_ext(L.u8(LR_RFLAGS)[l]) || !host::cresult_of(host::make_result(L, st, l, 0), &cr)
                ? 1u : 0u;
  }
}

__global__ void finish_total_c(const uint64_t* oc, const uint64_t* off, const uint32_t* rx, const uint32_t* roff,
                               uint32_t nl, uint32_t* total3) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const uint64_t t = nl ? off[nl - 1] + oc[nl - 1] : 0;
    total3[0] = (uint32_t)(t >> 32);
    total3[1] = (uint32_t)t;
    total3[2] = nl ? roff[nl - 1] + rx[nl - 1] : 0;
  }
}

__global__ void pack_outbox_c(SpaceView out, uint32_t nl, uint32_t S, const uint64_t* off, const uint32_t* peer_of_lane,
                              gr_cmsg* rec, gr_message* ext) {
  for (uint32_t l = io_tid(); l < nl; l += io_stride()) {
    uint32_t o = (uint32_t)(off[l] >> 32), eo = (uint32_t)off[l];
    const uint32_t peer = peer_of_lane[l];
    for (uint32_t j = 0; j < S; ++j)
      mailbox_records(out.at(j * nl + l), peer, j, [&](gr_cmsg cm, const gr_message* full) {
        if (full) {
          cm.flags = GR_CM_EXT;
          cm.aux = eo;
          ext[eo++] = *full;
        }
        rec[o++] = cm;
      });
  }
}

__global__ void pack_results_c(LaneBase L, StateBase st, const uint32_t* peer_of_lane, uint32_t nl,
                               const uint32_t* roff, gr_cresult* out, gr_peer_result* ext) {
  for (uint32_t l = io_tid(); l < nl; l += io_stride()) {
    const gr_peer_result pr = host::make_result(L, st, l, peer_of_lane[l]);
    gr_cresult c;
    // the same test as out_counts_c's rx
    if (!host::cresult_of(pr, &c) || host::result_needs_ext(L.u8(LR_RFLAGS)[l])) {
      c.flags = GR_CR_EXT;
      c.aux = roff[l];
      ext[roff[l]] = pr;
    }
    out[l] = c;
  }
}

// Does any mailbox of the space hold a message with cold fields (nonempty and
// without MB_UNIFORM)? One store per wave that finds one.
__global__ void cold_used(SpaceView v, uint32_t* flag) {
  const uint64_t n = (uint64_t)v.n_chunks * v.pc;
  for (uint64_t g = io_tid(); g < n; g += io_stride()) {
    const uint8_t c = v.at((uint32_t)g).cnt();
    const bool cold = mb_n(c) && !(c & MB_UNIFORM);
    if (__ballot(cold) && (threadIdx.x & 63) == 0) *flag = 1;
  }
}

// ---------------------------------------------------------------- wire path
// gr_step_wire: decoded raftpb.Message records (gpuraft_wire.h grw_message,
// grw_entry, in HBM from grw_decode_device) become gr_message records on the
// device: (ClusterID, To) -> engine slot through the gr_bind_nodes table, From
// -> the sender's remote slot through the slot's RID rows, entries -> their
// term runs. It replaces the transport's per-message handoff
// (internal/transport/tcp.go:416-426 -> MessageBatch.Unmarshal,
// raftpb/raft_optimized.go:1050) and the host packing of gr_message records.
struct NodeKey {
  uint64_t cluster = 0, node = 0;
  uint32_t peer = NOPOS, pad = 0;
};
__host__ __device__ inline uint32_t node_hash(uint64_t c, uint64_t n) {
  uint64_t x = c * 0x9E3779B97F4A7C15ull ^ (n + 0x632BE59BD9B4E019ull + (c << 6) + (c >> 2));
  x ^= x >> 31;
  x *= 0xBF58476D1CE4E5B9ull;
  return (uint32_t)(x ^ (x >> 29));
}
// Why a message stays with the host (gpuraft.h gr_wire_reason).
enum : uint8_t {
  WR_ROUTED = 0, WR_NO_PEER = 1, WR_NONMEMBER = 2, WR_SNAPSHOT = 3, WR_TYPE = 4, WR_RUNS = 5, WR_INDEX = 6
};

template <int S>
__global__ void route_wire(const grw_message* wm, uint32_t n, const grw_entry* we, uint64_t n_ents,
                           const NodeKey* nodes, uint32_t tcap, StateBase st, gr_message* out, uint32_t* flag,
                           uint8_t* why) {
  using Rw = Rows<S>;
  for (uint32_t i = io_tid(); i < n; i += io_stride()) {
    const grw_message m = wm[i];
    uint8_t w = WR_ROUTED;
    uint32_t peer = NOPOS;
    for (uint32_t h = node_hash(m.cluster_id, m.to) & (tcap - 1), probe = 0; probe < tcap;
         h = (h + 1) & (tcap - 1), ++probe) {
      const NodeKey k = nodes[h];
      if (k.peer == NOPOS) break;
      if (k.cluster == m.cluster_id && k.node == m.to) {
        peer = k.peer;
        break;
      }
    }
    uint32_t slot = GR_SLOT_NONE;
    if (peer == NOPOS) {
      w = WR_NO_PEER;
    } else {
      const uint64_t rb = h_rb(st.u64(SR_HDR)[peer]);
#pragma unroll
      for (int j = 0; j < S; ++j)
        if (slot == GR_SLOT_NONE && rb_kind(rb, (uint32_t)j) != GR_SLOT_EMPTY && st.u64(Rw::RID + j)[peer] == m.from)
          slot = (uint32_t)j;
      if (slot == GR_SLOT_NONE) w = WR_NONMEMBER;
    }
    if (w == WR_ROUTED && m.snapshot_host) w = WR_SNAPSHOT;
    if (w == WR_ROUTED && (m.type < 0 || m.type > GR_TIMEOUT_NOW)) w = WR_TYPE;
    gr_message r;
    memset(&r, 0, sizeof(r));
    if (w == WR_ROUTED) {
      // entries -> at most two term runs; a Replicate's entries must be the
      // consecutive indices LogIndex+1.. (raft.go:485-488), which the records imply
      uint32_t runs = 0, run2 = 0;
      uint64_t rt0 = 0, rt1 = 0;
      bool cc = false, seq = true;
      if ((uint64_t)m.first_entry + m.n_entries > n_ents) w = WR_RUNS;
      for (uint32_t k = 0; w == WR_ROUTED && k < m.n_entries; ++k) {
        const grw_entry en = we[m.first_entry + k];
        cc = cc || en.type == 1;  // raftpb.ConfigChangeEntry
        seq = seq && en.index == m.log_index + 1 + k;
        if (k == 0) {
          rt0 = en.term;
          runs = 1;
        } else if (en.term != (runs == 1 ? rt0 : rt1)) {
          if (runs == 2) w = WR_RUNS;
          runs = 2;
          run2 = k;
          rt1 = en.term;
        }
      }
      if (w == WR_ROUTED && m.type == GR_REPLICATE && !seq) w = WR_INDEX;
      r.peer = peer;
      r.slot = (uint8_t)slot;
      r.type = (uint8_t)m.type;
      // a forwarded Propose carrying a config change travels with the reject bit
      // (gpuraft.h, as Lane::propose forwards it)
      r.reject = (uint8_t)((m.reject ? 1 : 0) | (m.type == GR_PROPOSE && cc ? 1 : 0));
      r.n_runs = (uint8_t)runs;
      r.n_entries = m.n_entries;
      r.run2_offset = runs == 2 ? run2 : 0;
      r.term = m.term;
      r.log_index = m.log_index;
      r.log_term = m.log_term;
      r.commit = m.commit;
      r.hint = m.hint;
      r.hint_high = m.hint_high;
      r.run_term[0] = rt0;
      r.run_term[1] = rt1;
    }
    out[i] = r;
    flag[i] = w == WR_ROUTED ? 1u : 0u;
    why[i] = w;
  }
}
// Routed records to the front in wire order, unrouted indices after (pos =
// exclusive scan of flag); *n_routed = their count.
__global__ void keep_routed(const gr_message* rec, const uint32_t* flag, const uint32_t* pos, uint32_t n,
                            gr_message* out, uint32_t* unrouted, uint32_t* n_routed) {
  for (uint32_t i = io_tid(); i < n; i += io_stride()) {
    if (flag[i]) out[pos[i]] = rec[i];
    else unrouted[i - pos[i]] = i;
    if (i == n - 1) *n_routed = pos[i] + flag[i];
  }
}

// ---------------------------------------------------------------- side buffers
// Cross-GPU spaces (exchange.py Pipeline) send the hot region every pass and the
// cold fields only of the mailboxes that need them (no MB_UNIFORM), compacted
// into a fixed-capacity side buffer per chunk, so the all-to-all sizes are known
// without the host reading anything back. Per chunk: a 64-byte header (entry
// count) and `cap` entries of [u32 position in chunk][u32 count byte] + per
// message the 56 used bytes of its cold record (gr_layout.h Mailbox). A mailbox that does
// not fit gets MB_COLD_LOST in its (hot) count byte and its reader escalates
// CAPACITY.
constexpr uint32_t kSideHdr = 64;
__host__ __device__ inline uint32_t side_entry_bytes(uint32_t depth) { return 8 + depth * kColdUsed; }
__host__ __device__ inline uint64_t side_chunk_bytes(uint32_t depth, uint32_t cap) {
  return round256(kSideHdr + (uint64_t)cap * side_entry_bytes(depth));
}
// Copy the cold records (their kColdUsed bytes, 8-byte words) of the first n
// messages of mailbox mb into / out of entry e.
__host__ __device__ inline void cold_gather(const Mailbox& mb, uint32_t n, uint8_t* e) {
  for (uint32_t k = 0; k < n; ++k) {
    const uint64_t* src = reinterpret_cast<const uint64_t*>(mb.rec(k));
    uint64_t* dst = reinterpret_cast<uint64_t*>(e + 8 + k * kColdUsed);
    for (uint32_t w = 0; w < kColdUsed / 8; ++w) dst[w] = src[w];
  }
}
__host__ __device__ inline void cold_scatter(const Mailbox& mb, uint32_t n, const uint8_t* e) {
  for (uint32_t k = 0; k < n; ++k) {
    uint64_t* dst = reinterpret_cast<uint64_t*>(mb.rec(k));
    const uint64_t* src = reinterpret_cast<const uint64_t*>(e + 8 + k * kColdUsed);
    for (uint32_t w = 0; w < kColdUsed / 8; ++w) dst[w] = src[w];
  }
}
// One position of the pack: entry index idx (or >= cap: lost).
__host__ __device__ inline void side_put(const SpaceView& v, uint32_t g, uint8_t* side, uint32_t cap, uint32_t idx) {
  const Mailbox mb = v.at(g);
  const uint32_t cb = mb.cnt(), c = g / v.pc;
  if (idx >= cap) {
    mb.cnt() = (uint8_t)(cb | MB_COLD_LOST);
    return;
  }
  uint8_t* e = side + (uint64_t)c * side_chunk_bytes(v.depth, cap) + kSideHdr + (uint64_t)idx * side_entry_bytes(v.depth);
  reinterpret_cast<uint32_t*>(e)[0] = g - c * v.pc;
  reinterpret_cast<uint32_t*>(e)[1] = cb;
  cold_gather(mb, mb_n(cb), e);
}
__host__ __device__ inline bool needs_cold(uint32_t cb) { return mb_n(cb) && !(cb & MB_UNIFORM); }

// Pack the out space's cold fields into the side buffers (their counts zeroed
// before): one returning atomic per wave and chunk (a chunk is a multiple of 256
// positions, so a wave never spans two).
__global__ void side_pack(SpaceView v, uint8_t* side, uint32_t cap) {
  const uint64_t n = (uint64_t)v.n_chunks * v.pc;
  for (uint64_t g0 = (uint64_t)blockIdx.x * kIoBlock; g0 < n; g0 += (uint64_t)gridDim.x * kIoBlock) {
    const uint64_t g = g0 + threadIdx.x;
    const bool want = g < n && needs_cold(v.at((uint32_t)g).cnt());
    const uint64_t bm = __ballot(want);
    if (!bm) continue;
    const uint32_t lane = threadIdx.x & 63, first = (uint32_t)__ffsll((unsigned long long)bm) - 1;
    uint32_t base = 0;
    if (lane == first) {
      const uint32_t c = (uint32_t)(g / v.pc);
      base = atomicAdd(reinterpret_cast<uint32_t*>(side + (uint64_t)c * side_chunk_bytes(v.depth, cap)),
                       (uint32_t)__popcll(bm));
    }
    base = __shfl(base, (int)first);
    if (want) side_put(v, (uint32_t)g, side, cap, base + (uint32_t)__popcll(bm & ((1ull << lane) - 1)));
  }
}
// Unpack the received side buffers into the in space's cold chunks.
__global__ void side_unpack(SpaceView v, const uint8_t* side, uint32_t cap) {
  const uint64_t n = (uint64_t)v.n_chunks * cap;
  for (uint64_t t = io_tid(); t < n; t += io_stride()) {
    const uint32_t c = (uint32_t)(t / cap), idx = (uint32_t)(t % cap);
    const uint8_t* h = side + (uint64_t)c * side_chunk_bytes(v.depth, cap);
    const uint32_t cnt = *reinterpret_cast<const uint32_t*>(h);
    if (idx >= cnt) continue;
    const uint8_t* e = h + kSideHdr + (uint64_t)idx * side_entry_bytes(v.depth);
    const uint32_t pos = reinterpret_cast<const uint32_t*>(e)[0], cb = reinterpret_cast<const uint32_t*>(e)[1];
    cold_scatter(v.at(c * v.pc + pos), mb_n(cb), e);
  }
}

// ---------------------------------------------------------------- compact exchange
// The spread placement's all-to-all (exchange.py) in a compact
// form: per chunk a fixed-size buffer (fixed, so the all-to-all split sizes are
// known without the host reading anything back) that carries only the mailboxes
// with messages. A uniform mailbox whose messages repeat message 0's hot fields
// (one message, or a shared pair: gr_layout.h MB_SHARED -- the steady state's
// commit broadcast + proposal, and their two accepts) travels as a 12-byte
// record: its term word, the low 32 bits of its LogIndex (the high bits are the
// wave's, in the wave header), and its count byte with a 24-bit Commit offset
// (Replicates; |Commit - LogIndex| < 2^23). A mailbox outside that takes the full
// path. Every other mailbox with messages travels
// as a full side entry (hot fields of every message and their cold records). An
// empty mailbox costs one bit. Layout of a chunk's buffer (cx_layout):
//   header (kCxSub + 1) x 64 B: per record region one u32 counter of the
//     records taken (the packers' counters, records past the region's capacity
//     included), then the side entries taken, each counter on a 64-B line of
//     its own (kCxCtr words apart: atomics on one line serialise)
//   per 64 positions (a wave): u64 record mask, u64 lost mask, u32 first record,
//     u32 LogIndex high bits
//   records, structure of arrays over `cap`: u32 term word, u32 LogIndex low
//     bits, u32 count byte | Commit offset << 8. The capacity is split into
//     cx_regions() equal regions, and the pack's workgroup b takes its records
//     in region b % regions: one returning atomic per workgroup on its region's
//     counter (round 6: 1,465 workgroups queued on one counter word cost ~25 us
//     per 500k-group pass; regions balance, since every region gets every
//     regions-th workgroup of the chunk).
//   side entries (`scap`): u32 position, u32 count byte, u32 term word, u32 pad,
//     per message (u32 Commit offset, u32 pad, u64 LogIndex), then per message
//     the kColdUsed bytes of its cold record
// A mailbox that fits neither (records past `cap`, side entries past `scap`)
// reaches the receiver as lost (count 1 | MB_COLD_LOST, not uniform): its reader
// escalates CAPACITY at its first message, as with gr_space_side_pack.
// In the steady state of BASELINE config 4 at N = 8 a rank sends 4 chunks of
// 2 x 1M positions, half of them empty with the benchmark's leaders (replica 0:
// the follower-to-follower slots) and a third with leaders spread evenly:
// 4 x (cap x 12 B + 31k wave headers x 24 B + side entries) = 58 MB per pass at
// cap = 0.55 x positions, 70 MB at 0.7, against 328 MB for the hot regions
// (41 B per position). exchange.py sizes cap.
constexpr uint32_t kCxSub = 16, kCxCtr = 16, kCxHdr = (kCxSub + 1) * kCxCtr * 4, kCxWave = 24;
__host__ __device__ inline uint32_t cx_side_entry_bytes(uint32_t depth) { return 16 + depth * (16 + kColdUsed); }
struct CxLayout {
  uint64_t waves, cb, term, lo, cd, side, bytes;
  uint32_t nwv, cap, scap;
};
__host__ __device__ inline CxLayout cx_layout(uint32_t pc, uint32_t depth, uint32_t cap, uint32_t scap) {
  CxLayout L;
  L.nwv = pc / 64;
  L.cap = cap;
  L.scap = scap;
  L.waves = kCxHdr;
  L.term = round256(kCxHdr + (uint64_t)L.nwv * kCxWave);
  L.lo = L.term + round256(4ull * cap);
  L.cb = L.lo + round256(4ull * cap);  // count byte | Commit offset << 8
  L.cd = L.cb;
  L.side = L.cb + round256(4ull * cap);
  L.bytes = L.side + round256((uint64_t)scap * cx_side_entry_bytes(depth));
  return L;
}
// Record regions of a chunk of nwv wave groups: one per kCxRegionWgs pack
// workgroups (the pack's workgroups take kCxPackGroups wave groups each), at
// most kCxSub, at least one. A chunk's fill follows its replica pairs' position
// ranges (pair-major), and a region serves every regions-th workgroup, so its
// demand is its share of the chunk's within one workgroup per pair range: with
// kCxRegionWgs = 256 that is under 2.5 % of a region (exchange.py CX_MARGIN
// covers it), and a chunk of fewer than 512 workgroups has one region (exact).
constexpr uint32_t kCxPackPer = 8, kCxPackGroups = kCxPackPer * 4, kCxRegionWgs = 256;
__host__ __device__ inline uint32_t cx_regions(uint32_t nwv) {
  const uint32_t n = ((nwv + kCxPackGroups - 1) / kCxPackGroups) / kCxRegionWgs;
  return n < 1u ? 1u : (n > kCxSub ? kCxSub : n);
}
// Region r's first record and capacity: its share of the chunk's capacity in
// proportion to the pack workgroups it serves (workgroups b with b % regions
// == r), so that a capacity sized for every position's worst case holds it in
// every region.
__host__ __device__ inline void cx_region(uint32_t nwv, uint32_t cap, uint32_t r, uint32_t* off, uint32_t* rcap) {
  const uint32_t wgs = (nwv + kCxPackGroups - 1) / kCxPackGroups, n = cx_regions(nwv);
  const uint32_t per = wgs / n, extra = wgs % n;  // regions below `extra` serve one workgroup more
  const uint32_t before = r * per + (r < extra ? r : extra), mine = per + (r < extra ? 1u : 0u);
  const uint32_t w = wgs ? wgs : 1u;
  *off = (uint32_t)((uint64_t)cap * before / w);
  *rcap = (uint32_t)((uint64_t)cap * (before + mine) / w) - *off;
}
// Mailbox mb (count byte cb) travels as a uniform record: its hot fields are
// message 0's, and a Replicate's Commit offset fits 24 bits (*w: the record's
// third word).
// From the count byte and message 0's Commit offset (cd0).
__host__ __device__ inline bool cx_uniform_w3(uint32_t cb, uint32_t cd0, uint32_t* w) {
  const uint32_t n = mb_n(cb);
  if (!(n && (cb & MB_UNIFORM) && (n == 1 || mb_shared(cb)))) return false;
  if (cb & MB_RESP) {  // an accept has no Commit
    *w = cb;
    return true;
  }
  const uint32_t d = cd0 - 0x80000000u + 0x800000u;  // Commit - LogIndex + 2^23
  *w = cb | (d << 8);
  return (d >> 24) == 0;
}
__host__ __device__ inline bool cx_record_kind(const Mailbox& mb, uint32_t cb, uint32_t* w) {
  const uint32_t n = mb_n(cb);
  if (!(n && (cb & MB_UNIFORM) && (n == 1 || mb_shared(cb)))) return false;
  return cx_uniform_w3(cb, (cb & MB_RESP) ? 0u : mb.t32(0, MT_CDELTA), w);
}

// Pattern records (round 6): any other mailbox of at most three messages whose
// messages are a pass's steady or tick-pass traffic -- a leader's commit
// broadcasts, heartbeat and proposal ([Replicate, Heartbeat, Replicate]:
// broadcastHeartbeatMessage, raft.go:567-587, between the Replicates of
// handleLeaderReplicateResp and ProposeEntries; after a tick pass the staggered
// [Replicate, Replicate, Replicate] of two commit advances and a proposal), a
// follower's acks with its HeartbeatResp between them ([accept, HeartbeatResp,
// accept]: raft.go:923-931, 971-974), a uniform mailbox its writer did not
// share -- also travels as one 12-byte record instead of a full entry (16 + 72
// B per message), so a pass with ticks exchanges no more than a steady one.
// Every message must be one of a few canonical forms that the receiver
// rebuilds exactly:
//   Replicate: tag CX_R0C/R1C (compact, as uniform_tag gives) or CX_R0/R1 (the
//     general lane's full form: entry count 0 or 1, LogTerm = Term, one run at
//     Term), at the mailbox's anchor LogIndex A;
//   accept (ReplicateResp, flags 0): LogIndex A for the first, each later one
//     the previous one's plus 0 or 1 (one ack per Replicate received, the
//     staggered commit advances' Replicates repeat a LogIndex);
//   Heartbeat (flags 0): empty context (Hint = HintHigh = 0: no ReadIndex
//     pending); its Commit in the chain below (sendHeartbeatMessage:
//     min(match, committed), raft.go:548-563);
//   HeartbeatResp (flags 0): empty context;
// all at one term (the record's term word); Replicates and accepts do not mix.
// The Commits of the Replicates and heartbeats form a chain: the first one's
// is A + d0 - 2^16, each later one's the previous one's plus 0 or 1 (a commit
// advance per ack). With no Replicate or accept the first Commit is A.
// Third word: bits 0-1 the count (1..3), bits 2-3 clear (bit 3 = MB_UNIFORM
// marks the uniform kind), bits 4-12 one 3-bit code per message, bits 13-14
// the steps of messages 1 and 2 (of the Commit chain, or of the accepts'
// LogIndex chain), bits 15-31 d0. The receiver rebuilds a
// mailbox of Replicates only or accepts only as a uniform one (shared when its
// messages repeat message 0's hot fields, as MB_SHARED says: the readers take
// the same messages either way), any other as a full one. A mailbox that fits
// neither kind travels as a full entry.
enum CxCode : uint32_t { CX_R0C = 0, CX_R1C = 1, CX_R0 = 2, CX_R1 = 3, CX_ACC = 4, CX_HB = 5, CX_HBR = 6, CX_NONE = 7 };
constexpr uint32_t kCxPatStepShift = 13, kCxPatCdShift = 15, kCxPatCdBias = 1u << 16;
__host__ __device__ inline uint32_t cx_code_tag(uint32_t code) {  // the tag (type | flags << 8) a code stands for
  switch (code) {
    case CX_R0C: return GR_REPLICATE | ((uint32_t)MFL_COMPACT << 8);
    case CX_R1C: return GR_REPLICATE | ((uint32_t)(MFL_COMPACT | MFL_N1 | (1u << MFL_RUNS_SHIFT)) << 8);
    case CX_R0: return GR_REPLICATE;
    case CX_R1: return GR_REPLICATE | ((1u << MFL_RUNS_SHIFT) << 8);
    case CX_ACC: return GR_REPLICATE_RESP;
    case CX_HB: return GR_HEARTBEAT;
    case CX_HBR: return GR_HEARTBEAT_RESP;
    default: return 0xFFFFu;
  }
}
__host__ __device__ inline bool code_is_rep_full(uint32_t tag) {
  return tag == cx_code_tag(CX_R0) || tag == cx_code_tag(CX_R1);
}
// Classify mailbox mb (count byte cb) for the compact exchange: true when it
// travels as a record, with *w its third word, *li its anchor value and *anch
// whether the anchor's high bits must match the wave's (false for a record of
// HeartbeatResps alone, which has none).
__host__ __device__ inline bool cx_classify(const Mailbox& mb, uint32_t cb, uint32_t depth, uint32_t* w, uint64_t* li,
                                            bool* anch) {
  *anch = true;
  if (cx_record_kind(mb, cb, w)) {
    *li = mb.u64(0, MF_LOG_INDEX);
    return true;
  }
  const uint32_t n = mb_n(cb);
  const bool uni = (cb & MB_UNIFORM) != 0;
  if (!n || n > 3 || n > depth || (!uni && (cb & ~(uint32_t)MB_COUNT))) return false;
  uint32_t codes = 0, term = uni ? mb.mterm() : 0u, nacc = 0, steps = 0, d0 = 0;
  uint64_t a = 0, prevc = 0, prevl = 0;
  bool have_a = false, have_c = false, rep = false, acc = false, hbonly = true, ok = true;
  for (uint32_t k = 0; k < n && ok; ++k) {
    uint32_t tag, t;
    uint64_t commit = 0, hint = 0, hint_hi = 0;
    if (uni) {  // tag and term from the count byte and the term word (gr_layout.h)
      tag = Mailbox::uniform_tag(cb, k);
      t = term;
    } else {
      const uint32_t* r = reinterpret_cast<const uint32_t*>(mb.rec(k));
      tag = r[0] & 0xFFFFu;
      t = r[1];
      commit = reinterpret_cast<const uint64_t*>(r)[4];
      hint = reinterpret_cast<const uint64_t*>(r)[5];
      hint_hi = reinterpret_cast<const uint64_t*>(r)[6];
      if (k == 0) term = t;
      if (code_is_rep_full(tag)) {  // the full form: the fields the general lane writes
        const uint32_t ne = r[2], lt = r[4], rt0 = r[5];
        const bool one = tag == cx_code_tag(CX_R1);
        ok = ne == (one ? 1u : 0u) && lt == t && (!one || rt0 == t);
      }
    }
    ok = ok && t == term;
    uint32_t code = CX_NONE;
    for (uint32_t c = 0; c < CX_NONE; ++c) code = (code == CX_NONE && cx_code_tag(c) == tag) ? c : code;
    ok = ok && code != CX_NONE;
    if (!ok) break;
    bool carries = false;
    if (code <= CX_R1) {
      const uint64_t l = mb.log_index_at(k, cb);
      commit = commit_of(mb.cdelta_at(k, cb), l);
      ok = !acc && (!rep || l == a);
      if (!rep && !have_a) a = l;
      ok = ok && l == a;
      rep = have_a = true;
      hbonly = false;
      carries = true;
    } else if (code == CX_ACC) {  // LogIndex steps of 0 or 1 (an ack per Replicate, raft.go:971-974)
      const uint64_t l = mb.log_index_at(k, cb);
      ok = !rep && !have_c;
      if (nacc) {
        const uint64_t st = l - prevl;
        ok = ok && st <= 1u;
        steps |= (uint32_t)(st & 1u) << (k - 1);
      } else {
        a = l;
      }
      prevl = l;
      acc = have_a = true;
      hbonly = false;
      nacc++;
    } else if (code == CX_HB) {
      ok = !acc && hint == 0 && hint_hi == 0;
      carries = true;
    } else {  // CX_HBR
      ok = hint == 0 && hint_hi == 0;
    }
    if (ok && carries) {
      if (!have_c) {
        prevc = commit;
        have_c = true;
      } else {
        const uint64_t st = commit - prevc;
        ok = st <= 1u;
        steps |= (uint32_t)(st & 1u) << (k - 1);
        prevc = commit;
      }
    }
    codes |= code << (3 * k);
  }
  if (!ok) return false;
  // the first Commit relative to the anchor (the steps are the Commit chain's
  // when the mailbox carries Commits: accepts and Commits never mix)
  uint64_t first = 0;
  if (have_c) {
    uint64_t c0 = prevc;  // walk back the steps to the first Commit
    for (uint32_t k = n; k-- > 1;) c0 -= (steps >> (k - 1)) & 1u;
    first = c0;
  }
  if (have_c && !have_a) {  // heartbeats (and their acks) alone: the first Commit is the anchor
    a = first;
    have_a = true;
  }
  if (have_c) {
    const uint64_t dd = first - a + kCxPatCdBias;  // mod 2^64
    if (dd >= 2ull * kCxPatCdBias) return false;
    d0 = (uint32_t)dd;
  } else {
    d0 = kCxPatCdBias;
  }
  (void)hbonly;
  *anch = have_a;
  *li = have_a ? a : 0ull;
  *w = n | (codes << 4) | (steps << kCxPatStepShift) | (d0 << kCxPatCdShift);
  return true;
}
__host__ __device__ inline void cx_put_record(uint32_t term, uint64_t li, uint32_t w, uint8_t* buf, const CxLayout& L,
                                              uint32_t r) {
  reinterpret_cast<uint32_t*>(buf + L.term)[r] = term;
  reinterpret_cast<uint32_t*>(buf + L.lo)[r] = (uint32_t)li;
  reinterpret_cast<uint32_t*>(buf + L.cb)[r] = w;
}
// A record's term word: message 0's term (uniform mailboxes: the term word).
__host__ __device__ inline uint32_t cx_term_of(const Mailbox& mb, uint32_t cb) {
  return (cb & MB_UNIFORM) ? mb.mterm() : mb.t32(0, MT_TERM);
}
__host__ __device__ inline void cx_put_side(const Mailbox& mb, uint32_t cb, uint32_t pos, uint8_t* buf,
                                            const CxLayout& L, uint32_t depth, uint32_t x) {
  uint8_t* e = buf + L.side + (uint64_t)x * cx_side_entry_bytes(depth);
  const uint32_t n = mb_n(cb) < depth ? mb_n(cb) : depth;
  uint32_t* w = reinterpret_cast<uint32_t*>(e);
  w[0] = pos;
  w[1] = cb;
  w[2] = mb.mterm();
  w[3] = 0;
  for (uint32_t k = 0; k < n; ++k) {
    uint32_t* h = reinterpret_cast<uint32_t*>(e + 16 + 16 * k);
    h[0] = mb.t32(k, MT_CDELTA);
    h[1] = 0;
    *reinterpret_cast<uint64_t*>(h + 2) = mb.u64(k, MF_LOG_INDEX);
    const uint64_t* src = reinterpret_cast<const uint64_t*>(mb.rec(k));
    uint64_t* dst = reinterpret_cast<uint64_t*>(e + 16 + 16 * depth + kColdUsed * k);
    for (uint32_t q = 0; q < kColdUsed / 8; ++q) dst[q] = src[q];
  }
}
__host__ __device__ inline void cx_get_side(const Mailbox& mb, const uint8_t* e, uint32_t depth) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(e);
  const uint32_t cb = w[1], n = mb_n(cb) < depth ? mb_n(cb) : depth;
  mb.cnt() = (uint8_t)cb;
  mb.mterm() = w[2];
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t* h = reinterpret_cast<const uint32_t*>(e + 16 + 16 * k);
    mb.t32(k, MT_CDELTA) = h[0];
    mb.u64(k, MF_LOG_INDEX) = *reinterpret_cast<const uint64_t*>(h + 2);
    const uint64_t* src = reinterpret_cast<const uint64_t*>(e + 16 + 16 * depth + kColdUsed * k);
    uint64_t* dst = reinterpret_cast<uint64_t*>(mb.rec(k));
    for (uint32_t q = 0; q < kColdUsed / 8; ++q) dst[q] = src[q];
  }
}
// A pattern record (third word w, term t, anchor a) rebuilt into mailbox mb.
// Replicates only (all compact-equivalent) or accepts only: a uniform mailbox
// (count byte, term word, per message its hot fields; shared when they repeat
// message 0's). Otherwise a full one: the count byte, the term word, and per
// message the fields its readers read (gr_lane.h read_msg / decode_record,
// gr_tick.h): tag and term, LogIndex and Commit offset (Replicates; the full
// form's entry count, LogTerm and run term too), LogIndex (accepts), Commit and
// an empty context (heartbeats), an empty context (their acks).
__host__ __device__ inline void cx_get_pattern(const Mailbox& mb, uint32_t w, uint32_t t, uint64_t a) {
  const uint32_t n = w & 3u;
  uint32_t nrep = 0, nacc = 0, n1 = 0, allsame = 1, allone = 1;
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t code = (w >> (4 + 3 * k)) & 7u;
    nrep += code <= CX_R1;
    nacc += code == CX_ACC;
    n1 |= (uint32_t)(code == CX_R1 || code == CX_R1C) << k;
    if (k) {
      const uint32_t st = (w >> (kCxPatStepShift + k - 1)) & 1u;
      allsame &= st ^ 1u;
      allone &= st;
    }
  }
  uint64_t commit = a + (uint64_t)(w >> kCxPatCdShift) - kCxPatCdBias;
  mb.mterm() = t;
  if (nrep == n || nacc == n) {  // uniform (gr_layout.h MB_UNIFORM)
    const bool resp = nacc == n;
    const bool shared = n > 1 && (resp ? allone : allsame);  // MB_SHARED: accepts at +1, Replicates repeated
    mb.cnt() = (uint8_t)(n | MB_UNIFORM | (resp ? MB_RESP : 0u) | (shared ? MB_SHARED : 0u) |
                         (resp ? 0u : n1 << MB_N1_SHIFT));
    uint64_t li = a;
    for (uint32_t k = 0; k < (shared ? 1u : n); ++k) {
      const uint32_t st = k ? (w >> (kCxPatStepShift + k - 1)) & 1u : 0u;
      if (resp) li += st;
      else commit += st;
      mb.u64(k, MF_LOG_INDEX) = li;
      if (!resp) {
        uint32_t cd = 0;
        commit_delta(commit, a, &cd);
        mb.t32(k, MT_CDELTA) = cd;
      }
    }
    return;
  }
  mb.cnt() = (uint8_t)n;
  uint64_t ali = a;  // the accepts' LogIndex chain
  bool first_acc = true;
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t code = (w >> (4 + 3 * k)) & 7u;
    const uint32_t st = k ? (w >> (kCxPatStepShift + k - 1)) & 1u : 0u;
    if (nacc) {
      if (code == CX_ACC && !first_acc) ali += st;
    } else {
      commit += st;
    }
    mb.tag(k) = (uint16_t)cx_code_tag(code);
    mb.t32(k, MT_TERM) = t;
    if (code <= CX_R1) {
      uint32_t cd = 0;
      commit_delta(commit, a, &cd);
      mb.u64(k, MF_LOG_INDEX) = a;
      mb.t32(k, MT_CDELTA) = cd;
      const uint32_t ne = (code == CX_R1 || code == CX_R1C) ? 1u : 0u;
      mb.n(k) = ne;
      mb.t32(k, MT_LOG_TERM) = t;
      mb.t32(k, MT_RT0) = ne ? t : 0u;
    } else if (code == CX_ACC) {
      mb.u64(k, MF_LOG_INDEX) = ali;
      first_acc = false;
    } else if (code == CX_HB) {
      mb.u64(k, MF_COMMIT) = commit;
      mb.u64(k, MF_HINT) = 0;
      mb.u64(k, MF_HINT_HIGH) = 0;
    } else {
      mb.u64(k, MF_HINT) = 0;
      mb.u64(k, MF_HINT_HIGH) = 0;
    }
  }
}
// The wave header's effect on one position (lane): count byte and hot fields.
__host__ __device__ inline void cx_get_lane(const Mailbox& mb, const uint8_t* buf, const CxLayout& L, uint64_t mask,
                                            uint64_t lost, uint32_t base, uint32_t hi, uint32_t lane) {
  if ((mask >> lane) & 1ull) {
    const uint32_t r = base + (uint32_t)__builtin_popcountll(mask & ((1ull << lane) - 1));
    const uint32_t w = reinterpret_cast<const uint32_t*>(buf + L.cb)[r];
    if (!(w & MB_UNIFORM)) {  // a pattern record
      cx_get_pattern(mb, w, reinterpret_cast<const uint32_t*>(buf + L.term)[r],
                     ((uint64_t)hi << 32) | reinterpret_cast<const uint32_t*>(buf + L.lo)[r]);
      return;
    }
    mb.cnt() = (uint8_t)w;
    mb.mterm() = reinterpret_cast<const uint32_t*>(buf + L.term)[r];
    if (!(w & MB_RESP)) mb.t32(0, MT_CDELTA) = (w >> 8) - 0x800000u + 0x80000000u;
    mb.u64(0, MF_LOG_INDEX) = ((uint64_t)hi << 32) | reinterpret_cast<const uint32_t*>(buf + L.lo)[r];
  } else {
    mb.cnt() = ((lost >> lane) & 1ull) ? (uint8_t)(1u | MB_COLD_LOST) : (uint8_t)0;
  }
}

// Per-chunk record capacities (a chunk's fill depends on which replica pairs it
// carries: exchange.py) and the chunks' buffer offsets; kernel argument by value.
constexpr uint32_t kCxMaxChunks = 8;
struct CxCaps {
  uint32_t n, scap;
  uint32_t cap[kCxMaxChunks];
  uint64_t off[kCxMaxChunks + 1];
};
__host__ __device__ inline CxCaps cx_caps(uint32_t pc, uint32_t depth, uint32_t n, const uint32_t* caps,
                                          uint32_t scap) {
  CxCaps C{};
  C.n = n;
  C.scap = scap;
  C.off[0] = 0;
  for (uint32_t c = 0; c < n && c < kCxMaxChunks; ++c) {
    C.cap[c] = caps[c];
    C.off[c + 1] = C.off[c] + cx_layout(pc, depth, caps[c], scap).bytes;
  }
  return C;
}

// Pack: workgroup b of chunk c (blockIdx.y) takes kCxPackGroups consecutive
// wave groups (64 positions each), each of its four waves kCxPackPer of them in
// order (buffer headers zeroed before). A wave loads the hot fields of all its
// groups at once (count byte, term word, message 0's Commit offset and LogIndex:
// fixed addresses, no dependence on the count byte), classifies them (uniform
// mailboxes from those words; the rare non-uniform ones with their cold
// records, cx_classify) and counts records and side entries; the workgroup
// takes its record slots, then its side entries (its own plus the records past
// capacity), with one returning atomic each; then each wave writes its records,
// side entries and wave headers from the same registers. A wave's records are
// consecutive over its groups, in lane order. (Round 5 took the slots with a
// returning atomic per wave on one word per chunk: 360 us per 500k-group pass
// of one chunk, 47k waves queued on it; round 6's first cut, one group's loads
// at a time, 44 us.)
static_assert(kCxPackGroups == kCxPackPer * (kIoBlock / 64), "a pack workgroup is four waves");
__global__ __launch_bounds__(kIoBlock) void cx_pack(SpaceView v, uint8_t* cx, CxCaps C) {
  constexpr uint32_t nwave = kIoBlock / 64;
  const uint32_t c = blockIdx.y, nwv = v.pc / 64;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t g0 = blockIdx.x * kCxPackGroups + wave * kCxPackPer;
  const uint32_t cap = C.cap[c], scap = C.scap;
  const CxLayout L = cx_layout(v.pc, v.depth, cap, scap);
  uint8_t* buf = cx + C.off[c];
  __shared__ uint32_t s_rec[nwave], s_side[nwave], s_base[2];
  const uint32_t reg = blockIdx.x % cx_regions(nwv);
  uint32_t roff, rcap;
  cx_region(nwv, cap, reg, &roff, &rcap);
  // ---- every group's hot words in one batch (groups past the chunk: position 0's)
  uint32_t cb[kCxPackPer], cd[kCxPackPer], tw[kCxPackPer];
  uint64_t li[kCxPackPer];
#pragma unroll
  for (uint32_t q = 0; q < kCxPackPer; ++q) {
    const bool in = g0 + q < nwv;
    const Mailbox mb = v.at(c * v.pc + (in ? (g0 + q) * 64 + lane : 0u));
    cb[q] = mb.cnt();
    tw[q] = mb.mterm();
    cd[q] = mb.t32(0, MT_CDELTA);
    li[q] = mb.u64(0, MF_LOG_INDEX);
  }
#pragma unroll
  for (uint32_t q = 0; q < kCxPackPer; ++q) {  // every load issued before any value is used
    cb[q] = keep_value(cb[q]);
    tw[q] = keep_value(tw[q]);
    cd[q] = keep_value(cd[q]);
    li[q] = keep_value(li[q]);
  }
  uint32_t w3[kCxPackPer], hi[kCxPackPer];
  uint64_t recm = 0, msgm = 0;  // per group q: bit q
  uint32_t nrec = 0, nside = 0;
#pragma unroll
  for (uint32_t q = 0; q < kCxPackPer; ++q) {
    const bool in = g0 + q < nwv;
    const uint32_t b = in ? cb[q] : 0u;
    const bool msgs = mb_n(b) != 0;
    bool rec = false, anch = true;
    w3[q] = 0;
    if (msgs && (b & MB_UNIFORM)) {  // the uniform kind from the loaded words
      rec = cx_uniform_w3(b, cd[q], &w3[q]);
    }
    if (__ballot(msgs && !rec)) {  // pattern records (tick passes, unshared pairs): cx_classify
      if (msgs && !rec) {
        const Mailbox mb = v.at(c * v.pc + (g0 + q) * 64 + lane);
        uint64_t l = 0;
        rec = cx_classify(mb, b, v.depth, &w3[q], &l, &anch);
        if (rec) {
          li[q] = l;
          tw[q] = cx_term_of(mb, b);
        }
      }
    }
    const uint64_t any = __ballot(rec && anch);
    hi[q] = any ? (uint32_t)(__shfl((unsigned long long)li[q], __ffsll((unsigned long long)any) - 1) >> 32) : 0u;
    rec = rec && (!anch || (uint32_t)(li[q] >> 32) == hi[q]);
    recm |= (uint64_t)rec << q;
    msgm |= (uint64_t)msgs << q;
    nrec += (uint32_t)__popcll(__ballot(rec));
    nside += (uint32_t)__popcll(__ballot(msgs && !rec));
  }
  // ---- the workgroup's record slots and side entries
  if (lane == 0) s_rec[wave] = nrec;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t q = 0; q < nwave; ++q) t += s_rec[q];
    s_base[0] = t ? atomicAdd(reinterpret_cast<uint32_t*>(buf) + reg * kCxCtr, t) : 0u;
  }
  __syncthreads();
  uint32_t r = s_base[0];  // within the workgroup's region
  for (uint32_t q = 0; q < wave; ++q) r += s_rec[q];
  const uint32_t over = r >= rcap ? nrec : (r + nrec > rcap ? r + nrec - rcap : 0u);  // records past capacity
  if (lane == 0) s_side[wave] = nside + over;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t q = 0; q < nwave; ++q) t += s_side[q];
    s_base[1] = t ? atomicAdd(reinterpret_cast<uint32_t*>(buf) + kCxSub * kCxCtr, t) : 0u;
  }
  __syncthreads();
  uint32_t x0 = s_base[1];
  for (uint32_t q = 0; q < wave; ++q) x0 += s_side[q];
  // ---- records, side entries and wave headers
  const uint64_t below = (1ull << lane) - 1;
#pragma unroll
  for (uint32_t q = 0; q < kCxPackPer; ++q) {
    if (g0 + q >= nwv) break;  // wave-uniform
    const uint32_t g = g0 + q, pos = g * 64 + lane;
    const bool rec = (recm >> q) & 1u, msgs = (msgm >> q) & 1u;
    const uint64_t mask = __ballot(rec);
    const uint32_t ri = r + (uint32_t)__popcll(mask & below);
    const bool fits = rec && ri < rcap;  // past capacity: the group's last record lanes
    if (fits) cx_put_record(tw[q], li[q], w3[q], buf, L, roff + ri);
    const bool side = msgs && !fits;
    const uint64_t smask = __ballot(side);
    const uint32_t xi = x0 + (uint32_t)__popcll(smask & below);
    const bool sfits = side && xi < scap;
    if (sfits) {
      const Mailbox mb = v.at(c * v.pc + pos);
      cx_put_side(mb, mb.cnt(), pos, buf, L, v.depth, xi);
    }
    const uint64_t fmask = __ballot(fits), lost = __ballot(side && !sfits);
    if (lane == 0) {
      uint8_t* h = buf + L.waves + (uint64_t)g * kCxWave;
      reinterpret_cast<uint64_t*>(h)[0] = fmask;
      reinterpret_cast<uint64_t*>(h)[1] = lost;
      reinterpret_cast<uint32_t*>(h)[4] = roff + r;
      reinterpret_cast<uint32_t*>(h)[5] = hi[q];
    }
    r += (uint32_t)__popcll(mask);
    x0 += (uint32_t)__popcll(smask);
  }
}
// Unpack, part 1: every position's count byte and its record's hot fields.
// Each wave takes kCxUnpackPer consecutive wave groups of chunk blockIdx.y and
// issues their header loads, then all their record loads, as one batch each
// (round 5: one group per wave, two dependent round trips per group).
constexpr uint32_t kCxUnpackPer = 8, kCxUnpackGroups = kCxUnpackPer * (kIoBlock / 64);
__global__ __launch_bounds__(kIoBlock) void cx_unpack_waves(SpaceView v, const uint8_t* cx, CxCaps C) {
  const uint32_t c = blockIdx.y, nwv = v.pc / 64;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t g0 = blockIdx.x * kCxUnpackGroups + (threadIdx.x >> 6) * kCxUnpackPer;
  if (g0 >= nwv) return;  // wave-uniform; no barrier below
  const uint32_t cap = C.cap[c];
  const CxLayout L = cx_layout(v.pc, v.depth, cap, C.scap);
  const uint8_t* buf = cx + C.off[c];
  uint64_t mask[kCxUnpackPer], lost[kCxUnpackPer];
  uint32_t base[kCxUnpackPer], hi[kCxUnpackPer];
#pragma unroll
  for (uint32_t q = 0; q < kCxUnpackPer; ++q) {
    const uint8_t* h = buf + L.waves + (uint64_t)(g0 + q < nwv ? g0 + q : g0) * kCxWave;
    mask[q] = g0 + q < nwv ? reinterpret_cast<const uint64_t*>(h)[0] : 0ull;
    lost[q] = g0 + q < nwv ? reinterpret_cast<const uint64_t*>(h)[1] : 0ull;
    base[q] = reinterpret_cast<const uint32_t*>(h)[4];
    hi[q] = reinterpret_cast<const uint32_t*>(h)[5];
  }
  const uint64_t below = (1ull << lane) - 1;
  uint32_t tw[kCxUnpackPer], lo[kCxUnpackPer], w[kCxUnpackPer];
#pragma unroll
  for (uint32_t q = 0; q < kCxUnpackPer; ++q) {  // the records (index 0's when the lane has none)
    const bool has = cap && ((mask[q] >> lane) & 1ull);
    const uint32_t r = has ? base[q] + (uint32_t)__builtin_popcountll(mask[q] & below) : 0u;
    tw[q] = cap ? reinterpret_cast<const uint32_t*>(buf + L.term)[r] : 0u;
    lo[q] = cap ? reinterpret_cast<const uint32_t*>(buf + L.lo)[r] : 0u;
    w[q] = cap ? reinterpret_cast<const uint32_t*>(buf + L.cb)[r] : 0u;
  }
#pragma unroll
  for (uint32_t q = 0; q < kCxUnpackPer; ++q) {
    tw[q] = keep_value(tw[q]);
    lo[q] = keep_value(lo[q]);
    w[q] = keep_value(w[q]);
  }
#pragma unroll
  for (uint32_t q = 0; q < kCxUnpackPer; ++q) {
    if (g0 + q >= nwv) break;  // wave-uniform
    const Mailbox mb = v.at(c * v.pc + (g0 + q) * 64 + lane);
    if ((mask[q] >> lane) & 1ull) {
      const uint64_t a = ((uint64_t)hi[q] << 32) | lo[q];
      if (!(w[q] & MB_UNIFORM)) {
        cx_get_pattern(mb, w[q], tw[q], a);
      } else {
        mb.cnt() = (uint8_t)w[q];
        mb.mterm() = tw[q];
        if (!(w[q] & MB_RESP)) mb.t32(0, MT_CDELTA) = (w[q] >> 8) - 0x800000u + 0x80000000u;
        mb.u64(0, MF_LOG_INDEX) = a;
      }
    } else {
      mb.cnt() = ((lost[q] >> lane) & 1ull) ? (uint8_t)(1u | MB_COLD_LOST) : (uint8_t)0;
    }
  }
}
// Unpack, part 2 (after part 1): the side entries.
__global__ void cx_unpack_side(SpaceView v, const uint8_t* cx, CxCaps C) {
  const uint32_t scap = C.scap;
  const uint64_t n = (uint64_t)v.n_chunks * scap;
  for (uint64_t t = io_tid(); t < n; t += io_stride()) {
    const uint32_t c = (uint32_t)(t / scap), x = (uint32_t)(t % scap);
    const CxLayout L = cx_layout(v.pc, v.depth, C.cap[c], scap);
    const uint8_t* buf = cx + C.off[c];
    if (x >= reinterpret_cast<const uint32_t*>(buf)[kCxSub * kCxCtr]) continue;
    const uint8_t* e = buf + L.side + (uint64_t)x * cx_side_entry_bytes(v.depth);
    cx_get_side(v.at(c * v.pc + reinterpret_cast<const uint32_t*>(e)[0]), e, v.depth);
  }
}

// Zero the mailbox counts of chunk 0's first `positions` positions (the
// host-path inbox before encoding): one byte row untiled, the first 64 bytes of
// each tile with GR_TILE.
__global__ void clear_counts(SpaceView v, uint32_t positions) {
  for (uint32_t g = io_tid(); g < positions; g += io_stride()) v.at(g).cnt() = 0;
}

// ---- gr_peer records <-> SoA state rows: gr_load_groups/gr_sync_groups_to_host
// (slot range) and gr_load_peers/gr_sync_peers_to_host (slot list, the
// escalation hand-off of scattered groups). slots == nullptr: slot first + x.
constexpr uint32_t ERR_PEER = 1, ERR_SLOT = 2;

__global__ void check_peers(const gr_peer* in, const uint32_t* slots, uint32_t n, uint32_t S, uint32_t cap,
                            uint32_t* mark, uint32_t* err) {
  for (uint32_t x = io_tid(); x < n; x += io_stride()) {
    const gr_peer& g = in[x];
    if (g.n_runs > GR_K || g.read_index_count > GR_Q || (g.self_slot != GR_SLOT_NONE && g.self_slot >= S))
      atomicOr(err, ERR_PEER);
    // inMemory: markerIndex <= lastIndex + 1 (entries [marker, last])
    if (g.marker_index != 0 && g.marker_index > g.last_index + 1) atomicOr(err, ERR_PEER);
    if (slots) {  // in range and listed once, so the load is order-free
      if (slots[x] >= cap || atomicAdd(mark + slots[x], 1u) != 0) atomicOr(err, ERR_SLOT);
    }
  }
}

__global__ void peers_to_rows(const gr_peer* in, const uint32_t* slots, uint32_t first, uint32_t n, StateBase st,
                              uint32_t S) {
  const uint32_t n64 = rows_u64(S), n8 = rows_u8(S);
  for (uint32_t x = io_tid(); x < n; x += io_stride()) {
    const uint32_t p = slots ? slots[x] : first + x;
    const gr_peer& g = in[x];
    for (uint32_t r = 0; r < n64; ++r) st.u64(r)[p] = host::get_u64_row(g, r, S);
    for (uint32_t r = 0; r < n8; ++r) st.u8(r)[p] = host::get_u8_row(g, r, S);
  }
}

// `out` is zeroed first: fields with no row (padding, unused slots) read 0.
__global__ void rows_to_peers(StateBase st, const uint32_t* slots, uint32_t first, uint32_t n, uint32_t S,
                              gr_peer* out) {
  const uint32_t n64 = rows_u64(S), n8 = rows_u8(S);
  for (uint32_t x = io_tid(); x < n; x += io_stride()) {
    const uint32_t p = slots ? slots[x] : first + x;
    gr_peer& g = out[x];
    for (uint32_t r = 0; r < n64; ++r) host::set_u64_row(g, r, S, st.u64(r)[p]);
    host::resolve_sync(g, S, st.u64(SR_HDR)[p]);
    for (uint32_t r = 0; r < n8; ++r) host::set_u8_row(g, r, S, st.u8(r)[p]);
  }
}

// gr_notify_applied: one u64 row scattered over a slot list (slots checked on
// the host: in range, each listed once).
__global__ void set_row_u64(StateBase st, uint32_t row, const uint32_t* slots, const uint64_t* vals, uint32_t n) {
  for (uint32_t x = io_tid(); x < n; x += io_stride()) st.u64(row)[slots[x]] = vals[x];
}

// gr_compact_log: LogReader.Compact(index) (logreader.go:251-269) mirrored into
// entryLog.firstIndex()-1 (logentry.go:97-104). status: 0 ok, 1 ErrCompacted
// (index below firstIndex-1), 2 ErrUnavailable (index past the persisted lastIndex); only ok
// slots are written. H_GE_LO follows the new firstIndex-1.
template <int S>
__global__ void compact_rows(StateBase st, const uint32_t* slots, const uint64_t* idx, uint32_t n, int32_t* status,
                             uint32_t* refused) {
  for (uint32_t x = io_tid(); x < n; x += io_stride()) {
    const uint32_t p = slots[x];
    // LogReader.Compact checks its own range: markerIndex (firstIndex - 1 here)
    // and the persisted lastIndex, i.e. inMemory.savedTo (entries above it are
    // not in LogDB yet), not entryLog.lastIndex (logreader.go:251-269).
    const uint64_t i = idx[x], lo = st.u64(SR_LO)[p], last = st.u64(SR_SAVED_TO)[p];
    const int32_t rc = i < lo ? 1 : i > last ? 2 : 0;
    status[x] = rc;
    if (rc) {
      atomicOr(refused, 1u);
      continue;
    }
    st.u64(SR_LO)[p] = i;
    // The window forgets what the reference compacted away: runs wholly below
    // firstIndex-1 drop out and the run covering it starts there (term(i) is
    // LogReader's markerTerm), so the window never claims a term below it.
    const uint64_t h = st.u64(SR_HDR)[p];
    uint32_t nr = h_nruns(h);
    if (nr > GR_K) nr = GR_K;
    uint64_t rs[GR_K], rt[GR_K];  // oldest first
#pragma unroll
    for (int k = 0; k < GR_K; ++k) {
      const bool v = (uint32_t)k < nr;
      rs[k] = v ? st.u64(SR_RUN_START + run_row(nr, k))[p] : 0;
      rt[k] = v ? st.u64(SR_RUN_TERM + run_row(nr, k))[p] : 0;
    }
    uint32_t first = 0;  // last run starting at or below i
#pragma unroll
    for (int k = 1; k < GR_K; ++k)
      if ((uint32_t)k < nr && rs[k] <= i) first = k;
    uint32_t nn = nr;
    uint64_t ns[GR_K], nt[GR_K];
#pragma unroll
    for (int k = 0; k < GR_K; ++k) {
      ns[k] = rs[k];
      nt[k] = rt[k];
    }
    if (nr && rs[first] <= i) {  // drop runs [0, first), the covering run starts at i
      nn = nr - first;
#pragma unroll
      for (int k = 0; k < GR_K; ++k) {
        uint64_t a = 0, b = 0;
#pragma unroll
        for (int d = 0; d < GR_K; ++d)
          if ((uint32_t)d == (uint32_t)k + first) { a = rs[d]; b = rt[d]; }
        ns[k] = k == 0 ? i : a;
        nt[k] = b;
      }
#pragma unroll
      for (int k = 0; k < GR_K; ++k) {
        if ((uint32_t)k < nn) {
          st.u64(SR_RUN_START + run_row(nn, k))[p] = ns[k];
          st.u64(SR_RUN_TERM + run_row(nn, k))[p] = nt[k];
        }
      }
    }
    uint64_t newest = 0;
#pragma unroll
    for (int k = 0; k < GR_K; ++k)
      if ((uint32_t)k + 1 == nn) newest = ns[k];
    const bool ge = nn && newest >= i;
    // the run bits are cleared (the covering run may now start above committed);
    // with S > 6 those header bits are slot 7's rb field and stay
    const uint64_t rmask = has_run_bits((int)st.S) ? H_RUN_MASK : 0ull;
    st.u64(SR_HDR)[p] = h_make(h_state(h), h_self(h), nn, ge, h_flags(h), h_ric(h), h_rb(h)) & ~rmask;
  }
}

// gr_commit_update: entryLog.commitUpdate (logentry.go:325-335) with
// inMemory.savedLogTo / appliedLogTo (inmemory.go:92-139). status: 0 ok, 1 the
// reference panics (invalid applyto), 2 the term of stable_log_to is below the
// device window. Refused slots are not written.
__global__ void commit_rows(StateBase st, const uint32_t* slots, const gr_update_commit* uc, uint32_t n,
                            int32_t* status, uint32_t* refused) {
  for (uint32_t x = io_tid(); x < n; x += io_stride()) {
    const int32_t rc = host::commit_marks(st, slots[x], uc[x]);
    status[x] = rc;
    if (rc) atomicOr(refused, 1u);
  }
}

}  // namespace io
}  // namespace gr
