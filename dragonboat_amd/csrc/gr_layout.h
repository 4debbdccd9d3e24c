// gr_layout.h — device data layout of the gpuraft engine.
//
// Group state is structure-of-arrays in HBM, all in ONE allocation: row r of
// the u64 region is the array of one field over all engine slots, so a field
// address is base + r*8*cap + 8*p, with r a compile-time constant. The kernel
// therefore takes one base pointer and one row stride instead of ~70 array
// pointers (keeps the kernel argument small and in SGPRs).
//   u64 rows: scalar fields, the header word, term-run window [GR_K] x2,
//             remotes [S] x4, ReadIndex FIFO [GR_Q] x3
//   u8 rows:  ReadIndex FIFO [GR_Q] x2 (requester slot, ack bitmap)
// The header word packs every small field a lane tests (state, self slot,
// window run count, flags, FIFO count, and per remote slot state/active/kind):
// one 8-byte load instead of 5 + 3S byte loads.
// The term-run window is right-aligned: run r (0 = oldest) of n lives in row
// GR_K - n + r, so the newest run is always row GR_K - 1 and a lane reads it
// without first knowing n.
// Per-remote fields are [slot j][peer p], so a wave reading "match of slot j"
// for 64 consecutive peers reads 512 contiguous bytes.
//
// Messages live in "spaces" of mailboxes. A mailbox holds up to GR_C messages
// sent by one remote to one peer in one pass; message fields are SoA inside a
// chunk so a wave of lanes reading "message k of its mailbox" is coalesced.
// A space is n_chunks hot chunks followed by n_chunks cold chunks
// (pc = positions per chunk, a multiple of 64; depth = messages per mailbox):
//   hot chunk:  [cnt u8 x pc][term word u32 x pc] then for k < depth:
//               [commit offset u32 x pc][LogIndex u64 x pc]
//   cold chunk: for k < depth: [tag u16 x pc = type | flags << 8][term u32][n u32][run2 u32]
//               [log term u32][run term 0 u32][run term 1 u32][Commit u64][Hint u64][HintHigh u64] (each x pc)
// A uniform mailbox (MB_UNIFORM: the lean lane's steady-state compact Replicates
// or accepts, one term) lives in the hot chunk alone: 5 B plus 12 B per message.
// An exchange between GPUs moves the hot region always and the cold region only
// when some mailbox lacks the bit (gr_space_cold_used).
// Terms travel as 32 bits: a message whose term, log term or entry-run terms
// reach 2^32 never enters a mailbox (the sender escalates GR_ESC_WIDE_TERM;
// a host-encoded inbox marks it MT_WIDE and the receiver escalates there), so
// every value read back is exact. Indexes, commit and ReadIndex contexts stay 64-bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gpuraft.h"

namespace gr {

constexpr uint32_t NOPOS = 0xFFFFFFFFu;

// ---------------------------------------------------------------- state rows
enum U64Row : uint32_t {
  SR_TERM = 0, SR_VOTE, SR_COMMITTED, SR_APPLIED, SR_LAST_INDEX, SR_LO, SR_LEADER_ID, SR_LTT,
  SR_NODE_ID, SR_ETICK, SR_HTICK, SR_RETIMEOUT, SR_ETIMEOUT, SR_HTIMEOUT, SR_ENTRY_UB,
  SR_SAVED_TO, SR_MARKER, SR_LOG_APPLIED,  // inMemory.savedTo / markerIndex, entryLog.applied (§8f-4)
  SR_HDR,                          // the header word (below); 18: phys_row (GR_PAIR) pairs it with SR_TERM
  SR_RUN_START,                    // + row, right-aligned (run_row)
  SR_RUN_TERM = SR_RUN_START + GR_K,  // + r
  SR_REMOTE = SR_RUN_TERM + GR_K,     // remote rows start; see below
};
template <int S>
struct Rows {
  static constexpr uint32_t MATCH = SR_REMOTE;        // + j
  static constexpr uint32_t NEXT = MATCH + S;         // + j
  static constexpr uint32_t SNAP = NEXT + S;          // + j
  static constexpr uint32_t RID = SNAP + S;           // + j
  static constexpr uint32_t RI_INDEX = RID + S;       // + q
  static constexpr uint32_t RI_LO = RI_INDEX + GR_Q;  // + q
  static constexpr uint32_t RI_HI = RI_LO + GR_Q;     // + q
  static constexpr uint32_t NU64 = RI_HI + GR_Q;
  // u8 rows (after the u64 region)
  static constexpr uint32_t B_RIFROM = 0;             // + q
  static constexpr uint32_t B_RIACK = B_RIFROM + GR_Q;// + q
  static constexpr uint32_t NU8 = B_RIACK + GR_Q;
};
// Tile width of the tiled layouts (GR_TILE): 2^GR_TILE_SHIFT slots / positions.
// 256 (a workgroup's four waves share each row segment: 2 KB per u64 row)
// measured 0.1149 vs 0.1171 ms per 1M x 3 pass against 64, A/B in one call.
#ifndef GR_TILE_SHIFT
#define GR_TILE_SHIFT 8
#endif
constexpr uint32_t kTileW = 1u << GR_TILE_SHIFT, kTileM = kTileW - 1;
__host__ __device__ inline uint32_t pad_cap(uint32_t n) { return (n + kTileM) & ~kTileM; }
__host__ __device__ inline uint32_t rows_u64(uint32_t S) { return SR_REMOTE + 4 * S + 3 * GR_Q; }
__host__ __device__ inline uint32_t rows_u8(uint32_t) { return 2 * GR_Q; }
// row of run r (0 = oldest) of a window of n runs (right-aligned)
__host__ __device__ inline uint32_t run_row(uint32_t n, uint32_t r) { return GR_K - n + r; }

// ---------------------------------------------------------------- header word
//   bits 0-1 state, 2-5 self slot (15 = none), 6-8 n_runs, 9 H_GE_LO (the newest
//   run starts at or above firstIndex-1), 10-17 flags (GR_F_* and the device
//   bits below), 18-20 ReadIndex FIFO count, 24 + 5j remote slot j:
//   state (2 bits), active (1), kind (2) -- the `rb` word of gr_lane.h.
constexpr uint32_t H_SELF_SHIFT = 2, H_NRUNS_SHIFT = 6, H_GE_LO_BIT = 9, H_FLAGS_SHIFT = 10, H_RIC_SHIFT = 18,
                   H_REM_SHIFT = 24;
constexpr uint32_t H_SELF_NONE = 15;
__host__ __device__ inline uint32_t h_state(uint64_t h) { return (uint32_t)h & 3u; }
__host__ __device__ inline uint32_t h_self(uint64_t h) {
  const uint32_t s = (uint32_t)(h >> H_SELF_SHIFT) & 15u;
  return s == H_SELF_NONE ? GR_SLOT_NONE : s;
}
__host__ __device__ inline uint32_t h_nruns(uint64_t h) { return (uint32_t)(h >> H_NRUNS_SHIFT) & 7u; }
__host__ __device__ inline bool h_gelo(uint64_t h) { return (h >> H_GE_LO_BIT) & 1u; }
__host__ __device__ inline uint32_t h_flags(uint64_t h) { return (uint32_t)(h >> H_FLAGS_SHIFT) & 0xFFu; }
__host__ __device__ inline uint32_t h_ric(uint64_t h) { return (uint32_t)(h >> H_RIC_SHIFT) & 7u; }
__host__ __device__ inline uint64_t h_rb(uint64_t h) { return h >> H_REM_SHIFT; }
__host__ __device__ inline uint64_t h_make(uint32_t state, uint32_t self, uint32_t nruns, bool gelo, uint32_t flags,
                                           uint32_t ric, uint64_t rb) {
  const uint32_t s4 = self >= 15u ? H_SELF_NONE : self;
  return (uint64_t)(state & 3u) | ((uint64_t)s4 << H_SELF_SHIFT) | ((uint64_t)(nruns & 7u) << H_NRUNS_SHIFT) |
         ((uint64_t)(gelo ? 1u : 0u) << H_GE_LO_BIT) | ((uint64_t)(flags & 0xFFu) << H_FLAGS_SHIFT) |
         ((uint64_t)(ric & 7u) << H_RIC_SHIFT) | (rb << H_REM_SHIFT);
}
// Sync bits (S <= 3; above rb): bit H_NX_SHIFT + j says next[j] == lastIndex + 1
// and the NEXT row of slot j is stale; H_MS_BIT says match[self] == lastIndex and
// the MATCH row of the self slot is stale. Those are a steady-state leader's
// values (appendEntries advances its own remote, raft.go:643-654; every send in
// the Replicate state moves next to lastIndex + 1, remote.go:120-128), so the lean
// lane keeps them in the header instead of loading and storing 4 of its 6 remote
// rows per pass. Every other writer of lastIndex or of the remote rows first
// materialises the rows and clears the bits (Lane::store); the tick lane only
// reads them; host conversion resolves them (host::resolve_sync).
// H_MP_SHIFT + j (round 4) says match[j] == lastIndex - 2 for a slot j other
// than self, and its MATCH row is stale. In the pipelined steady state a pass's
// acks are for the entry proposed two passes earlier (a Replicate crosses one
// pass boundary to the follower, its ack another back), so after the acks
// (remote.tryUpdate, raft.go:1205-1227) and this pass's proposal
// (appendEntries :643-654) every follower's match is lastIndex - 2 again: a
// steady leader loads and stores none of its MATCH rows either.
constexpr uint32_t H_NX_SHIFT = 56, H_MS_BIT = 59, H_MP_SHIFT = 40;
constexpr uint64_t H_SYNC_MASK = (7ull << H_NX_SHIFT) | (1ull << H_MS_BIT) | (7ull << H_MP_SHIFT);
__host__ __device__ constexpr bool has_sync_bits(int S) { return S <= 3; }
__host__ __device__ inline bool h_nx(uint64_t h, uint32_t j) { return (h >> (H_NX_SHIFT + j)) & 1u; }
__host__ __device__ inline bool h_ms(uint64_t h) { return (h >> H_MS_BIT) & 1u; }
__host__ __device__ inline bool h_mp(uint64_t h, uint32_t j) { return (h >> (H_MP_SHIFT + j)) & 1u; }
// Run bits (S <= 6; above rb and the sync bits): H_RTT says the window's newest
// run has the current term, H_RLC that it starts at or below committed. Both
// hold in steady state (the leader's term's run began before the commit point),
// and then every index at or above committed is in the newest run at the
// current term: the lean lane tests the bits instead of loading the run's two
// rows. They are summaries (the rows stay exact): set only with at least one
// run; every writer of term, committed or the window recomputes or clears them.
constexpr uint32_t H_RTT_BIT = 60, H_RLC_BIT = 61;
constexpr uint64_t H_RUN_MASK = (1ull << H_RTT_BIT) | (1ull << H_RLC_BIT);
__host__ __device__ constexpr bool has_run_bits(int S) { return S <= 6; }
__host__ __device__ inline uint64_t run_bits(uint32_t nruns, uint64_t newest_start, uint64_t newest_term,
                                             uint64_t term, uint64_t committed) {
  if (!nruns) return 0;
  return (newest_term == term ? 1ull << H_RTT_BIT : 0ull) | (newest_start <= committed ? 1ull << H_RLC_BIT : 0ull);
}
// per-slot fields of rb (5 bits per slot: state(2) active(1) kind(2))
__host__ __device__ inline uint32_t rb_state(uint64_t rb, uint32_t j) { return (uint32_t)(rb >> (5 * j)) & 3u; }
__host__ __device__ inline uint32_t rb_active(uint64_t rb, uint32_t j) { return (uint32_t)(rb >> (5 * j + 2)) & 1u; }
__host__ __device__ inline uint32_t rb_kind(uint64_t rb, uint32_t j) { return (uint32_t)(rb >> (5 * j + 3)) & 3u; }
__host__ __device__ inline uint64_t rb_with(uint64_t rb, uint32_t j, uint32_t off, uint32_t width, uint32_t v) {
  const uint64_t m = ((1ull << width) - 1) << (5 * j + off);
  return (rb & ~m) | (((uint64_t)v << (5 * j + off)) & m);
}
__host__ __device__ inline uint64_t state_bytes(uint32_t S, uint32_t cap) {
  return (uint64_t)cap * (8ull * rows_u64(S) + rows_u8(S));
}

// GR_TILE = 1: the rows are tiled by kTileW slots (256, one workgroup): tile t
// holds every row of its slots, row-major inside the tile, so a workgroup's
// fields are one contiguous block instead of ~30 separate row streams (24 MB
// apart at 1M x 3). GR_TILE = 0: plain rows over all slots.
#ifndef GR_TILE
#define GR_TILE 1
#endif
// GR_PAIR = 1: inside a tile, the u64 rows every steady-state lane reads come
// in interleaved pairs, (term, header) and (committed, lastIndex): a lane's two
// fields of a pair are adjacent, so each pair loads and stores as one 16-byte
// access. Physical rows 0..3 hold the pairs; the other rows follow in order.
#ifndef GR_PAIR
#define GR_PAIR 0
#endif
__host__ __device__ constexpr uint32_t phys_row(uint32_t r) {
#if GR_PAIR
  return r == 0 ? 0u : r == 18 ? 1u : r == 2 ? 2u : r == 4 ? 3u  // SR_TERM, SR_HDR, SR_COMMITTED, SR_LAST_INDEX
         : 4u + r - (r > 0) - (r > 2) - (r > 4) - (r > 18);
#else
  return r;
#endif
}
template <class T>
struct TileRow {  // row `row` of a tiled region with `nrows` rows per tile
  T* b;
  uint32_t row, nrows;
  __host__ __device__ inline T& operator[](uint64_t p) const {
#if GR_PAIR
    if (sizeof(T) == 8) {
      const uint32_t ph = phys_row(row);
      if (ph < 4)
        return b[(((p >> GR_TILE_SHIFT) * nrows + (ph & ~1u)) * kTileW + 2 * (p & kTileM)) + (ph & 1u)];
      return b[((p >> GR_TILE_SHIFT) * nrows + ph) * kTileW + (p & kTileM)];
    }
#endif
    return b[((p >> GR_TILE_SHIFT) * nrows + row) * kTileW + (p & kTileM)];
  }
};
struct StateBase {
  uint8_t* base;
  uint32_t cap;  // padded, multiple of 64
  uint32_t S;
#if GR_TILE
  __host__ __device__ inline TileRow<uint64_t> u64(uint32_t row) const {
    return {reinterpret_cast<uint64_t*>(base), row, rows_u64(S)};
  }
  __host__ __device__ inline TileRow<uint8_t> u8(uint32_t row) const {
    return {base + 8ull * cap * rows_u64(S), row, rows_u8(S)};
  }
#else
  __host__ __device__ inline uint64_t* u64(uint32_t row) const {
    return reinterpret_cast<uint64_t*>(base) + (uint64_t)row * cap;
  }
  __host__ __device__ inline uint8_t* u8(uint32_t row) const {
    return base + 8ull * cap * rows_u64(S) + (uint64_t)row * cap;
  }
#endif
};

// ---------------------------------------------------------------- lane rows
// Per-pass arrays indexed by lane: local inputs and results.
enum LaneU64Row : uint32_t {
  LR_RI_LO = 0, LR_RI_HI, LR_RAND, LR_APPEND_FROM,
  LR_RTR_INDEX,                         // + q
  LR_RTR_LO = LR_RTR_INDEX + GR_Q,      // + q
  LR_RTR_HI = LR_RTR_LO + GR_Q,         // + q
  LR_NU64 = LR_RTR_HI + GR_Q,
};
enum LaneU32Row : uint32_t { LR_TICKS = 0, LR_QTICKS, LR_PROPOSE, LR_ESC_ITEM, LR_LANE_PEER, LR_LWORD, LR_FWD_ENTRIES,
                             LR_NU32 };
enum LaneU8Row : uint32_t { LR_LFLAGS = 0, LR_RFLAGS, LR_ESC_REASON, LR_PROP_RESULT, LR_RTR_COUNT, LR_FWD_COUNT,
                            LR_NU8 };
__host__ __device__ inline uint64_t lane_bytes(uint32_t S, uint32_t lcap) {
  // + in_pos / out_pos route tables [S][lcap] u32 each
  return (uint64_t)lcap * (8ull * LR_NU64 + 4ull * LR_NU32 + LR_NU8 + 8ull * S);
}
struct LaneBase {
  uint8_t* base;
  uint32_t lcap;
  uint32_t S;
  __host__ __device__ inline uint64_t* u64(uint32_t row) const {
    return reinterpret_cast<uint64_t*>(base) + (uint64_t)row * lcap;
  }
  __host__ __device__ inline uint32_t* u32(uint32_t row) const {
    return reinterpret_cast<uint32_t*>(base + 8ull * LR_NU64 * lcap) + (uint64_t)row * lcap;
  }
  __host__ __device__ inline uint8_t* u8(uint32_t row) const {
    return base + (8ull * LR_NU64 + 4ull * LR_NU32) * lcap + (uint64_t)row * lcap;
  }
  __host__ __device__ inline uint32_t* in_pos() const {
    return reinterpret_cast<uint32_t*>(base + (8ull * LR_NU64 + 4ull * LR_NU32 + LR_NU8) * lcap);
  }
  __host__ __device__ inline uint32_t* out_pos() const { return in_pos() + (uint64_t)S * lcap; }
};
constexpr uint8_t LF_READ_INDEX = 0x01;
constexpr uint8_t LF_PROPOSE_CC = 0x02;
// LR_LWORD: a lane's local inputs packed for the lean lane (4 bytes instead
// of 13): bits 0-15 the ProposeEntries count, bits 17-24 the QuiescedTick
// count, bit 16 set when there is anything else (ReadIndex, config change,
// ticks, or a count that does not fit), which the lean lane hands over.
// With bit 16 set, bit 26 (LW_TICKONLY) says the word still holds everything
// the tick lane takes (gr_tick.h: no proposal, no QuiescedTick, no config
// change): the Tick count in bits 17-24 and the ReadIndex flag in bit 25, so
// that lane reads one word instead of four rows.
constexpr uint32_t LW_OTHER = 0x10000u;
constexpr uint32_t LW_QT_SHIFT = 17, LW_QT_MAX = 0xFFu;
constexpr uint32_t LW_TICK_SHIFT = 17, LW_TICK_MAX = 0xFFu, LW_RI = 1u << 25, LW_TICKONLY = 1u << 26;
__host__ __device__ inline uint32_t local_word(uint32_t ticks, uint32_t qticks, uint32_t propose, uint32_t lflags) {
  const bool other = ticks || lflags || propose > 0xFFFFu || qticks > LW_QT_MAX;
  if (!other) return propose | (qticks << LW_QT_SHIFT);
  if (!qticks && !propose && !(lflags & ~(uint32_t)LF_READ_INDEX) && ticks <= LW_TICK_MAX)
    return LW_OTHER | LW_TICKONLY | (ticks << LW_TICK_SHIFT) | ((lflags & LF_READ_INDEX) ? LW_RI : 0u);
  return LW_OTHER;
}
// Device-internal bits of the header's flags byte (never visible in gr_peer.flags:
// gr_host.h masks them; GR_F_* use bits 0-2). They let the lean lane test one
// bit instead of loading or rewriting 8-byte fields:
//   F_LTT    leaderTransferTarget != 0
//   F_ETZ    electionTick == 0
//   F_LSLOT  0, or s + 1 for a remote slot s < 7 with remote_id[s] == leaderID
// Every device write of those fields updates the bits (Lane::store, FastLane).
constexpr uint32_t F_PUBLIC = 0x07u;
constexpr uint32_t F_LTT = 0x80u;
constexpr uint32_t F_ETZ = 0x40u;
constexpr uint32_t F_LSLOT_SHIFT = 3, F_LSLOT = 0x38u;
// H_GE_LO: the newest run starts at or above firstIndex-1, so every index at
// or above it is inside the log window and the lean lane never needs
// firstIndex-1 (lo).
// The result record's propose_first is not stored: ProposeEntries is the last
// item of a pass, so it is last_index - propose_entries + 1 after the pass.
constexpr uint8_t RF_ESCALATED = 0x01;
constexpr uint8_t RF_PROPOSE = 0x02;
constexpr uint8_t RF_READY = 0x04;
constexpr uint8_t RF_APPEND = 0x08;
constexpr uint8_t RF_FORWARDED = 0x10;  // forwarded Propose batches appended: LR_FWD_COUNT, LR_FWD_ENTRIES
constexpr uint8_t RF_HARDSTATE = 0x20;  // term or vote changed (pb.Update.State differs)

// ---------------------------------------------------------------- message spaces
enum U64Field : uint32_t { MF_LOG_INDEX = 0, MF_COMMIT = 1, MF_HINT = 2, MF_HINT_HIGH = 3, MF_NUM_U64 = 4 };
enum T32Field : uint32_t { MT_TERM = 0, MT_LOG_TERM = 1, MT_RT0 = 2, MT_RT1 = 3, MT_CDELTA = 4, MT_NUM = 5 };
constexpr uint8_t MFL_REJECT = 0x01;
constexpr uint8_t MFL_RUNS_SHIFT = 1;     // bits 1..2: n_runs
constexpr uint8_t MFL_WIDE_COMMIT = 0x08; // Replicate: Commit in MF_COMMIT (else MT_CDELTA)
// Compact Replicate (the steady state): LogTerm == Term, at most one entry,
// whose term is Term, narrow Commit. Only type, flags, Term, LogIndex and the
// Commit offset are written; MFL_N1 gives the entry count (0 or 1).
constexpr uint8_t MFL_COMPACT = 0x10;
constexpr uint8_t MFL_N1 = 0x20;
// The mailbox count byte: bits 0-2 the count (GR_C + 1 marks an overflowed
// host-encoded mailbox). Bit 3 (MB_UNIFORM): at most kUniformMax messages, all
// compact Replicates (bit 4 clear) or all non-reject ReplicateResps (bit 4 set),
// all at the mailbox's term word; bits 5.. give MFL_N1 of message 0, 1, 2. Such
// a mailbox stores only the hot fields (the term word, and LogIndex + Commit
// offset per message): readers rebuild every tag and term from the count byte,
// so they touch neither the per-message tags and terms nor the cold chunk. Only
// the lean lane writes uniform mailboxes; every other writer stores all fields.
constexpr uint8_t MB_COUNT = 0x07, MB_UNIFORM = 0x08, MB_RESP = 0x10;
// Shared uniform mailboxes (MB_UNIFORM | MB_SHARED; the count is then bits 0-1):
// the steady state's two messages per mailbox repeat each other's hot fields, so
// only message 0's are stored. Compact Replicates: every message has message
// 0's LogIndex and Commit offset (a commit broadcast and the proposal after it,
// both at the leader's old lastIndex: makeReplicateMessage, raft.go:474-498);
// accepts: message k has LogIndex = message 0's + k (the acks of those two
// Replicates, LogIndex + entries, raft.go:971-974). A shared Replicate mailbox
// stores 12 bytes less per extra message, a shared ack mailbox 8. Readers take
// the count from mb_n and the fields from Mailbox::log_index_at / cdelta_at.
constexpr uint8_t MB_SHARED = 0x04;
__host__ __device__ inline uint32_t mb_n(uint32_t cb) { return (cb & MB_UNIFORM) ? (cb & 3u) : (cb & MB_COUNT); }
__host__ __device__ inline bool mb_shared(uint32_t cb) {
  return (cb & (MB_UNIFORM | MB_SHARED)) == (MB_UNIFORM | MB_SHARED);
}
// On a mailbox without MB_UNIFORM, bit 4 means its cold fields did not fit the
// exchange's side buffer (gr_io.h side_pack): a reader escalates CAPACITY at its
// first message instead of reading them (cross-GPU spaces only).
constexpr uint8_t MB_COLD_LOST = 0x10;
constexpr uint32_t MB_N1_SHIFT = 5, kUniformMax = 3;
// A Replicate's Commit travels as a 32-bit offset from its LogIndex when
// |Commit - LogIndex| < 2^31 (always, unless a follower lags by 2^31 entries);
// otherwise in full with MFL_WIDE_COMMIT. Both decode exactly.
__host__ __device__ inline bool commit_delta(uint64_t commit, uint64_t log_index, uint32_t* cd) {
  const uint64_t d = commit - log_index + 0x80000000ull;  // mod 2^64
  if (d >> 32) return false;
  *cd = (uint32_t)d;
  return true;
}
__host__ __device__ inline uint64_t commit_of(uint32_t cd, uint64_t log_index) {
  return log_index + (uint64_t)cd - 0x80000000ull;
}
constexpr uint8_t MT_WIDE = 0xFF;      // type of a host-encoded message whose terms do not fit 32 bits
__host__ __device__ inline bool wide_term(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
  return ((a | b | c | d) >> 32) != 0;
}

__host__ __device__ inline uint32_t space_pad_positions(uint32_t positions) {
  return (positions + kTileM) & ~kTileM;
}
constexpr uint32_t kHotH = 5;    // bytes per position, hot chunk header: count + term word
constexpr uint32_t kHotK = 12;   // bytes per position per message, hot chunk: Commit offset + LogIndex
// ... cold chunk: one 64-byte record per position and message (the fields of
// gr_layout.h Mailbox, 56 bytes used). The cold fields belong to the irregular
// traffic (heartbeats and their acks, rejects, full Replicates), whose lanes are
// scattered over the chunk: a record keeps a message's cold fields in one line
// instead of one line per field (10 with the field-major layout it replaced).
constexpr uint32_t kColdK = 64, kColdUsed = 56;
__host__ __device__ inline uint64_t round256(uint64_t b) { return (b + 255u) & ~(uint64_t)255u; }
// A space's mailbox depth (1..GR_C) fixes its chunk sizes: spaces that cross
// xGMI use the depth the steady state needs (2).
// GR_TILE: a chunk's positions are tiled by kTileW (pc is a multiple of it): tile
// t of the hot region holds the counts and hot fields of its kTileW positions, the
// same SoA order as an untiled chunk of kTileW positions; the cold region alike.
__host__ __device__ inline uint64_t tile_hot_bytes(uint32_t depth) { return (uint64_t)kTileW * (kHotH + kHotK * depth); }
__host__ __device__ inline uint64_t tile_cold_bytes(uint32_t depth) { return (uint64_t)kTileW * kColdK * depth; }
__host__ __device__ inline uint64_t space_hot_chunk_bytes_pc(uint32_t pc, uint32_t depth = GR_C) {
  return round256((uint64_t)pc * (kHotH + kHotK * depth));  // = pc/64 tiles when tiled
}
__host__ __device__ inline uint64_t space_cold_chunk_bytes_pc(uint32_t pc, uint32_t depth = GR_C) {
  return round256((uint64_t)pc * kColdK * depth);
}
__host__ __device__ inline uint64_t space_chunk_bytes_pc(uint32_t pc, uint32_t depth = GR_C) {
  return space_hot_chunk_bytes_pc(pc, depth) + space_cold_chunk_bytes_pc(pc, depth);
}

// Streaming access for the lean lane: every state and message byte of a pass
// is touched once per pass and the working set is far above the caches, so its
// loads carry the nontemporal hint: 0.148 vs 0.156 ms per 1M x 3 pass, A/B in
// one call (GR_NT=0 builds without). Nontemporal stores (GR_NT_ST=1) measured
// 0.152: the lane's stores stay default.
#ifndef GR_NT
#define GR_NT 1
#endif
template <class T>
__host__ __device__ inline T ntld(const T& r) {
#if GR_NT && defined(__HIP_DEVICE_COMPILE__)
  return __builtin_nontemporal_load(&r);
#else
  return r;
#endif
}
#ifndef GR_NT_ST
#define GR_NT_ST 0
#endif
// The value as an opaque definition (device code): an empty asm that reads and
// writes it, so code that uses a loaded value only under a condition cannot make
// the load conditional (a branch around a load made the compiler wait for it
// before the next one: one round trip per slot and message). Issue a batch of
// loads, then pass each value through this. Identity in host builds.
template <class T>
__host__ __device__ inline T keep_value(T v) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(v));
#endif
  return v;
}

template <class T>
__host__ __device__ inline void ntst(T& r, T v) {
#if GR_NT_ST && defined(__HIP_DEVICE_COMPILE__)
  __builtin_nontemporal_store(v, &r);
#else
  r = v;
#endif
}

struct Mailbox {
  uint8_t* hot;   // the chunk's hot part
  uint8_t* cold;  // ... and its cold part
  uint32_t local;
  uint32_t pc;
  // hot:  [count u8][term word u32], then per message [Commit offset u32][LogIndex u64]
  //       (each field x pc positions)
  // cold: per message, a 64-byte record per position (message-major):
  //       [tag u16][pad u16][term u32][n u32][run2 u32][log term u32][rt0 u32][rt1 u32][pad u32]
  //       [Commit u64][Hint u64][HintHigh u64][pad u64]
  __host__ __device__ inline uint8_t* hk(uint32_t k) const { return hot + (kHotH + (uint64_t)k * kHotK) * pc; }
  __host__ __device__ inline uint8_t* rec(uint32_t k) const { return cold + ((uint64_t)k * pc + local) * kColdK; }
  __host__ __device__ inline uint8_t& cnt() const { return hot[local]; }
  __host__ __device__ inline uint32_t& mterm() const { return reinterpret_cast<uint32_t*>(hot + pc)[local]; }
  __host__ __device__ inline uint8_t& type(uint32_t k) const { return rec(k)[0]; }
  __host__ __device__ inline uint8_t& flags(uint32_t k) const { return rec(k)[1]; }
  // type | flags << 8 in one access (little-endian)
  __host__ __device__ inline uint16_t& tag(uint32_t k) const { return *reinterpret_cast<uint16_t*>(rec(k)); }
  __host__ __device__ inline uint32_t& n(uint32_t k) const { return reinterpret_cast<uint32_t*>(rec(k))[2]; }
  __host__ __device__ inline uint32_t& run2(uint32_t k) const { return reinterpret_cast<uint32_t*>(rec(k))[3]; }
  __host__ __device__ inline uint32_t& t32(uint32_t k, uint32_t f) const {
    if (f == MT_CDELTA) return reinterpret_cast<uint32_t*>(hk(k))[local];
    if (f == MT_TERM) return reinterpret_cast<uint32_t*>(rec(k))[1];
    // MT_LOG_TERM, MT_RT0, MT_RT1: record words 4, 5, 6
    return reinterpret_cast<uint32_t*>(rec(k))[4 + (f - MT_LOG_TERM)];
  }
  __host__ __device__ inline uint64_t& u64(uint32_t k, uint32_t f) const {
    if (f == MF_LOG_INDEX) return reinterpret_cast<uint64_t*>(hk(k) + 4ull * pc)[local];
    // MF_COMMIT, MF_HINT, MF_HINT_HIGH: record u64 words 4, 5, 6
    return reinterpret_cast<uint64_t*>(rec(k))[4 + (f - MF_COMMIT)];
  }
  // Tag and term of message k given the mailbox's count byte `cb` (MB_UNIFORM:
  // rebuilt from the count byte and the term word, else the stored fields).
  __host__ __device__ inline uint32_t tag_at(uint32_t k, uint32_t cb) const {
    return (cb & MB_UNIFORM) ? uniform_tag(cb, k) : (uint32_t)tag(k);
  }
  __host__ __device__ inline uint32_t term_at(uint32_t k, uint32_t cb) const {
    return (cb & MB_UNIFORM) ? mterm() : t32(k, MT_TERM);
  }
  // LogIndex and Commit offset of message k given the count byte (shared
  // mailboxes: derived from message 0's, which is all they store)
  __host__ __device__ inline uint64_t log_index_at(uint32_t k, uint32_t cb) const {
    if (k && mb_shared(cb)) return u64(0, MF_LOG_INDEX) + ((cb & MB_RESP) ? (uint64_t)k : 0ull);
    return u64(k, MF_LOG_INDEX);
  }
  __host__ __device__ inline uint32_t cdelta_at(uint32_t k, uint32_t cb) const {
    return t32(k && mb_shared(cb) ? 0u : k, MT_CDELTA);
  }
  __host__ __device__ static inline uint32_t uniform_tag(uint32_t cb, uint32_t k) {
    if (cb & MB_RESP) return GR_REPLICATE_RESP;  // flags 0: an accept
    const bool n1 = (cb >> (MB_N1_SHIFT + k)) & 1u;
    return GR_REPLICATE | ((uint32_t)(MFL_COMPACT | (n1 ? (MFL_N1 | (1u << MFL_RUNS_SHIFT)) : 0u)) << 8);
  }
};

struct SpaceView {
  uint8_t* base;
  uint32_t n_chunks;
  uint32_t pc;
  uint64_t hot_bytes;   // per chunk; the hot region is n_chunks * hot_bytes at base
  uint64_t cold_bytes;  // per chunk; the cold region follows the hot region
  uint32_t depth;  // messages per mailbox (1..GR_C); emitting more escalates CAPACITY
  // ONE: the space is known to have one chunk (loopback spaces; the lean
  // kernel's RT_LOOPBACK instance): no chunk division or branch.
  template <bool ONE = false>
  __host__ __device__ inline Mailbox at(uint32_t gpos) const {
    const uint32_t c = (ONE || n_chunks == 1) ? 0u : gpos / pc;  // one chunk (loopback spaces): no division
    Mailbox m;
    m.hot = base + (uint64_t)c * hot_bytes;
    m.cold = base + (uint64_t)n_chunks * hot_bytes + (uint64_t)c * cold_bytes;
    m.local = gpos - c * pc;
#if GR_TILE
    const uint32_t t = m.local >> GR_TILE_SHIFT;
    m.hot += t * tile_hot_bytes(depth);
    m.cold += t * tile_cold_bytes(depth);
    m.local &= kTileM;
    m.pc = kTileW;
#else
    m.pc = pc;
#endif
    return m;
  }
};

// Stats partials: one row of NSTAT u64 per workgroup, owned by that workgroup.
enum StatField : uint32_t {
  ST_PASSES = 0, ST_LEADER_COMMITS = 1, ST_FOLLOWER_COMMITS = 2, ST_ESCALATIONS = 3,
  ST_MSGS_IN = 4, ST_MSGS_OUT = 5, ST_LEADER_MSGS_IN = 6, ST_LEADER_MSGS_OUT = 7,
  ST_REPLICATE_ENTRIES = 8, ST_BAILED = 9, NSTAT = 16
};
// Per-lane counters of one pass (reduced per workgroup into the stats rows).
// "leader" = the lane ended the pass as leader; entries = sum of n over the
// Replicate messages the lane handled (the units of SURVEY.md §8d).
struct LaneStats {
  uint32_t leader_commit = 0, follower_commit = 0, escalated = 0;
  uint32_t msgs_in = 0, msgs_out = 0, leader_in = 0, leader_out = 0, entries = 0;
  uint32_t bailed = 0;  // left the lean kernels (stepped by the tick or general lane)
};

// Route modes: where lane i reads (dir 0) / writes (dir 1) the mailbox of
// remote slot j.
//   RT_IDENTITY: j*n_lanes + i (slot-major, so a wave touches consecutive mailboxes)
//   RT_TABLE:    in_pos/out_pos tables [S][lcap] in the lane block
//   RT_AFFINE:   replica-major populations (lane i = r*G + g): base[dir][r][j] + g,
//                base NOPOS = no mailbox. Detected by gr_bind_routes from the
//                tables; saves the 8*S bytes of route reads per lane.
//   RT_LOOPBACK: the one-space replica-major loopback (all replicas of a group in
//                this engine, route_r blocks of route_g lanes): in = j*n + i,
//                out = r*n + j*G + g, none when j == r or j >= route_r. No table
//                load, so the mailbox counts load in the first round.
constexpr uint8_t RT_IDENTITY = 0, RT_TABLE = 1, RT_AFFINE = 2, RT_LOOPBACK = 3;

// Wave hints: one byte per wave of lanes (device-resident path), what the
// wave's lanes were at the end of the previous pass, so the lean lane can issue
// that role's loads with its first round (gr_fast.h). 0 = mixed or idle.
// Follower hints carry the leader's slot in bits 2..; leader hints carry the
// self slot in bits 2-4 and WH_SYNC when every lane's remote rows were in sync
// (H_NX for every member slot and H_MS), so no NEXT row or own MATCH row is loaded.
// WH_RUNS: every lane's run bits were set, so no lane loads the newest run's rows.
constexpr uint32_t WH_ROLE = 3, WH_LEADER = 1, WH_FOLLOWER = 2, WH_SLOT_SHIFT = 2, WH_SYNC = 0x20, WH_RUNS = 0x40;
// Bytes per hint set: a byte per wave, padded so each set starts 16-byte
// aligned and a workgroup's four hints load as one scalar dword (gr_kernels.h).
__host__ __device__ inline uint64_t hint_stride(uint32_t cap) { return ((uint64_t)cap / 64 + 16) & ~(uint64_t)15; }
// The lean kernel (FL_* of gr_fast.h) that steps a wave with hint h.
__host__ __device__ inline int wave_kernel(uint32_t h, int S) {
  if ((h & WH_ROLE) == WH_LEADER && S <= 3) return 1;  // FL_LEADER
  if ((h & WH_ROLE) == WH_FOLLOWER) return 2;          // FL_FOLLOWER
  return 0;                                            // FL_ANY
}

// Kernel argument (small, passed by value, lives in SGPRs).
// Lane i steps peer lane_peer[i] (identity when has_lane_peer == 0).
struct StepParams {
  StateBase st;
  LaneBase ln;
  SpaceView in, out;
  uint64_t* stats;     // [gridDim.x][NSTAT] or nullptr
  uint8_t* hints;      // [n_lanes / 64] wave hints (WH_*) as the pass started, or nullptr
  uint8_t* hints_out;  // ... the next pass's (written by the kernel that steps the wave)
  const uint32_t* route_base;  // RT_AFFINE: [2][GR_SMAX][GR_SMAX]
  uint64_t max_entry_size;
  uint32_t n_lanes;
  uint32_t route_g;    // RT_AFFINE / RT_LOOPBACK: groups per replica block
  uint32_t route_r;    // RT_LOOPBACK: replica blocks
  uint8_t has_locals;
  uint8_t has_lane_peer;
  uint8_t route_mode;
  uint8_t split;       // follower-hinted waves go to the FL_FOLLOWER instance (gr_kernels.h)
  uint8_t route_wu;    // route_g % 64 == 0: replica_of is wave-uniform
  // host-side launch choice (gr_kernels.h launch): passes of at most this many
  // workgroups run as one fused kernel (gr_small_kernel)
  uint32_t small_blocks;
  // GR_WAVE_CLOCK (profiling, gr_engine.hip): per general-kernel wave a record of
  // kWaveClockWords u64 (start and end clock, lanes, messages in, escalations,
  // leader messages), or nullptr
  uint64_t* wclock;
  // lanes handed to the general kernel go to lists keyed by handler class
  // (gr_kernels.h general_bin) instead of by role and workgroup
  uint8_t bin_general;
  // the tail hint (gr_kernels.h kTailAll): one word of host-visible pinned
  // memory the general kernel writes after each split pass (did the role
  // instances have work, how many lanes the general kernel stepped), which the
  // host reads, unsynchronised, to size the next launches' grids; nullptr: off
  uint32_t* tail_hint;
  // which tail launches a pass makes (gr_kernels.h TailPlan): 0 = from the
  // tail hint; 1 or 3 = the role instances always (round 4's schedule); 2 =
  // never (the general kernel steps the listed waves and every hand-over).
  // GR_TAIL_MODE at gr_create.
  uint8_t tail_mode;
  // set by the launcher for the steady kernel of a pass whose role instances do
  // not run: its non-steady lanes go to the retry lists (gr_kernels.h GM_RETRY)
  uint8_t no_roles;
  // the tick lane's staged inputs (TickStage): one record per tick-list entry,
  // written by the steady kernel (nullptr: the tick lane loads everything itself)
  uint64_t* tick_stage;
  uint32_t pass_tag;  // the launch number: a record of this pass carries it
};
// A tick-list entry's staged inputs (round 5): the fields the steady kernel
// loads for every lane of a wave that is not steady (coalesced: the wave's
// quiesced lanes load the same lines), so the tick lane reads one 32-byte record
// instead of a header, electionTick, locals word and S count bytes scattered
// over as many lines. Words: header, electionTick, locals word | pass tag << 32,
// the S in-mailbox count bytes.
constexpr uint32_t kTickStageWords = 4;
constexpr uint32_t kWaveClockWords = 8;
// The wave's clock for GR_WAVE_CLOCK phase marks (0 when off, and in host builds).
__host__ __device__ inline uint64_t lane_clock(const StepParams& kp) {
#if defined(__HIP_DEVICE_COMPILE__)
  return kp.wclock ? wall_clock64() : 0ull;
#else
  (void)kp;
  return 0ull;
#endif
}

// Route mode as a compile-time parameter of the lean kernel instances
// (gr_kernels.h): RM_ANY reads StepParams::route_mode at run time; an instance
// built for RT_LOOPBACK or RT_AFFINE has no route branches, so every address of
// the lane's first load round is known before any load is issued (with the run
// time switch the compiler kept the route arithmetic behind a wait for the
// state loads: two dependent memory rounds instead of one).
constexpr int RM_ANY = -1;
// The replica block of lane i (RT_LOOPBACK / RT_AFFINE: lane i = r * route_g + g).
// StepParams::route_wu (route_g a multiple of 64): a wave's lanes share r, so it
// is one scalar division per wave instead of a vector division per lane.
__host__ __device__ inline uint32_t replica_of(const StepParams& kp, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (kp.route_wu) return __builtin_amdgcn_readfirstlane(i) / kp.route_g;
#endif
  return i / kp.route_g;
}
// Every route of lane i at once (in[j], out[j] for j < S): the lane's replica
// block and group are divided out once, not once per slot and direction.
template <int S, int RM = RM_ANY>
__host__ __device__ inline void routes_of(const StepParams& kp, uint32_t i, uint32_t* in, uint32_t* out) {
  const uint32_t mode = RM == RM_ANY ? (uint32_t)kp.route_mode : (uint32_t)RM;
  if (mode == RT_LOOPBACK || mode == RT_AFFINE) {
    const uint32_t r = replica_of(kp, i), g = i - r * kp.route_g;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      if (mode == RT_LOOPBACK) {
        const bool none = (uint32_t)j == r || (uint32_t)j >= kp.route_r;
        const uint32_t n = kp.route_r * kp.route_g;
        in[j] = none ? NOPOS : j * n + i;
        out[j] = none ? NOPOS : r * n + j * kp.route_g + g;
      } else {
        const uint32_t bi = kp.route_base[(0 * GR_SMAX + r) * GR_SMAX + j];
        const uint32_t bo = kp.route_base[(1 * GR_SMAX + r) * GR_SMAX + j];
        in[j] = bi == NOPOS ? NOPOS : bi + g;
        out[j] = bo == NOPOS ? NOPOS : bo + g;
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < S; ++j) {
    in[j] = mode == RT_TABLE ? kp.ln.in_pos()[(uint64_t)j * kp.ln.lcap + i] : j * kp.n_lanes + i;
    out[j] = mode == RT_TABLE ? kp.ln.out_pos()[(uint64_t)j * kp.ln.lcap + i] : j * kp.n_lanes + i;
  }
}
__host__ __device__ inline uint32_t route_of(const StepParams& kp, uint32_t dir, uint32_t j, uint32_t i) {
  if (kp.route_mode == RT_TABLE)
    return (dir ? kp.ln.out_pos() : kp.ln.in_pos())[(uint64_t)j * kp.ln.lcap + i];
  if (kp.route_mode == RT_LOOPBACK) {
    const uint32_t r = i / kp.route_g;
    if (j == r || j >= kp.route_r) return NOPOS;
    const uint32_t n = kp.route_r * kp.route_g;
    return dir ? r * n + j * kp.route_g + (i - r * kp.route_g) : j * n + i;
  }
  if (kp.route_mode == RT_AFFINE) {
    const uint32_t r = i / kp.route_g, g = i - r * kp.route_g;
    const uint32_t b = kp.route_base[(dir * GR_SMAX + r) * GR_SMAX + j];
    return b == NOPOS ? NOPOS : b + g;
  }
  return j * kp.n_lanes + i;
}

}  // namespace gr
