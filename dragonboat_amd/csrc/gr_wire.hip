// gr_wire.hip — libgrwire.so: the raft wire codec (MessageBatch / Message /
// Entry marshal and unmarshal) as HIP passes for gfx950, C-ABI in
// include/gpuraft_wire.h. SURVEY.md §8f-2.
//
// The work is byte parsing: varints, tag dispatch and bounds checks. It is
// HBM/latency bound with no MFMA. Structure:
//
// decode (MessageBatch.Unmarshal, raft_optimized.go:1050-1202)
//   1. walk_frames   one wave per frame walks the top-level fields through a
//                    4 KiB LDS window loaded with coalesced 16-B reads: message
//                    spans (into a scratch slot per 2 frame bytes, so no scan is
//                    needed first), DeploymentId/SourceAddress/BinVer, the first
//                    walk error and whether messageCount panics.
//      (frames of >= 4 segments on average first run spec_segments: one wave
//      per 8 KiB segment walks a speculative chain that walk_frames adopts)
//   2. scan          exclusive sum of messages per frame -> first_msg.
//   3. decode_msgs   one lane per message: every Message field (last wins),
//                    entries validated (colfer), entry count, Snapshot span.
//   4. scan          exclusive sum of entries per message -> first_entry.
//   5. decode_ents   one lane per entry; the first entry's lane writes its
//                    message's Entry records (map_ents builds the map).
//   6. finish        one lane per frame: status = first error in wire order.
// encode (MessageBatch.MarshalTo, raft.pb.go:1929-1958)
//   1. size_msgs     one lane per message: Message.Size() and its field size.
//   2. scan (u64)    message positions in the stream of message fields.
//   3. frame_sizes   one lane per frame: MessageBatch.Size(); scan -> offsets.
//   4. write_msgs    one lane per message writes tag, length and Message bytes.
//   5. write_tails   one lane per frame writes DeploymentId/SourceAddress/BinVer.
#include <hip/hip_runtime.h>

#pragma clang diagnostic ignored "-Wunused-value"

#include <algorithm>
#include <cstdlib>
#include <vector>
#include <cstring>
#include <mutex>
#include <new>

#include "gpuraft.h"
#include "gpuraft_wire.h"
#include "gr_scan.h"  // hand-written exclusive scan (shared with the engine)

namespace grw {

using u8 = uint8_t;
using u32 = uint32_t;
using i32 = int32_t;
using u64 = uint64_t;
using i64 = int64_t;

__device__ __forceinline__ i64 wrap_add(i64 a, i64 b) { return (i64)((u64)a + (u64)b); }

// Snapshot{}.MarshalTo (raft.pb.go:1696-1735, empty Membership :1589-1594).
__constant__ u8 kZeroSnap[12] = {0x12, 0x00, 0x18, 0x00, 0x20, 0x00, 0x28, 0x00, 0x32, 0x02, 0x08, 0x00};

// ------------------------------------------------------------ byte readers --

// Per-lane reader over buf[0, len): one aligned 16-B load per 16 bytes walked,
// byte loads only for a chunk that crosses the buffer's ends.
struct Rd {
  const u8* buf;
  u64 len;
  u64 cbase;   // absolute offset of the cached 16-B chunk, ~0 = none
  u64 lo, hi;  // the chunk, as two words: bytes are taken by shifts (an indexed
               // read of a vector would put the chunk in scratch memory)
  const uint4* lds = nullptr;  // optional block-staged copy of buf[llo, lhi), 16-B aligned
  u64 llo = 0, lhi = 0;
  __device__ Rd(const u8* b, u64 l) : buf(b), len(l), cbase(~0ull), lo(0), hi(0) {}
  __device__ __forceinline__ u8 at(u64 a) {  // a < len
    u64 base = a & ~15ull;
    if (base != cbase) {
      uint4 c;
      const u8* p = buf + base;
      if (base >= llo && base < lhi) {
        c = lds[(base - llo) >> 4];
      } else if ((((uintptr_t)p) & 15) == 0 && base + 16 <= len) {
        // Cached load: the next chunk of the same message is in the same line
        // (a nontemporal load refetched each line once per 16 B: 2.5x slower).
        c = *(const uint4*)p;
      } else {  // a chunk crossing the buffer's ends: a rolled byte loop, no call
        u64 x = 0, y = 0;
#pragma unroll 1
        for (u32 k = 0; k < 16 && base + k < len; ++k) {
          u64 v = p[k];
          if (k < 8) x |= v << (8 * k); else y |= v << (8 * (k - 8));
        }
        c = make_uint4((u32)x, (u32)(x >> 32), (u32)y, (u32)(y >> 32));
      }
      lo = (u64)c.y << 32 | c.x;
      hi = (u64)c.w << 32 | c.z;
      cbase = base;
    }
    u32 o = (u32)a & 15;
    u64 m = 0ull - (u64)(o >> 3);  // all ones for the high word: arithmetic, not a select
    return (u8)((lo ^ ((lo ^ hi) & m)) >> ((o & 7) * 8));
  }
};

// One frame's bytes through an LDS window, walked by a whole wave in lockstep
// (every lane computes the same offsets, so branches stay uniform).
constexpr int kWin = 4096;
struct Win {
  u8* lds;
  const u8* buf;
  u64 buf_len;
  u64 lo, hi;
  __device__ __forceinline__ void load(u64 at) {
    __syncthreads();
    lo = at & ~15ull;
    hi = lo + kWin < buf_len ? lo + kWin : buf_len;
    for (int k = threadIdx.x; k < kWin / 16; k += 64) {
      u64 a = lo + (u64)k * 16;
      uint4 v = make_uint4(0, 0, 0, 0);
      const u8* p = buf + a;
      if (a + 16 <= buf_len && (((uintptr_t)p) & 15) == 0) {
        v = *(const uint4*)p;
      } else if (a < buf_len) {
        u8 t[16];
        for (int j = 0; j < 16; ++j) t[j] = (a + j < buf_len) ? p[j] : 0;
        memcpy(&v, t, 16);
      }
      ((uint4*)lds)[k] = v;
    }
    if (threadIdx.x == 0) ((uint4*)lds)[kWin / 16] = make_uint4(0, 0, 0, 0);
    __syncthreads();
  }
  __device__ __forceinline__ u8 at(u64 a) {  // a < buf_len
    if (a < lo || a >= hi) load(a);
    return lds[a - lo];
  }
  // Bytes a..a+3 (zeros past the buffer) as one wave-uniform scalar: two
  // aligned LDS dword reads and a funnel shift, then readfirstlane, so the
  // walk's branches are scalar.
  __device__ __forceinline__ u32 peek4(u64 a) {
    if (a < lo || a + 4 > hi) {
      if (a < lo || hi < buf_len || a >= hi) load(a);
    }
    u32 o = (u32)(a - lo);
    const u32* d = (const u32*)lds;
    u64 pair = (u64)d[o >> 2] | ((u64)d[(o >> 2) + 1] << 32);
    return __builtin_amdgcn_readfirstlane((u32)(pair >> (8 * (o & 3))));
  }
};

// Checked varint (raft_optimized.go:658-671) on a frame-relative cursor i over
// [0, l); `R` maps frame offsets to bytes.
template <class R>
__device__ __forceinline__ int rd_varint(R& r, u64 base, i64 l, i64& i, u64& v) {
  v = 0;
  for (u32 shift = 0;; shift += 7) {
    if (shift >= 64) return GRW_E_INT_OVERFLOW;
    if (i >= l) return GRW_E_UNEXPECTED_EOF;
    u8 b = r.at(base + (u64)i);
    i++;
    v |= (u64)(b & 0x7F) << shift;
    if (b < 0x80) break;
  }
  return GRW_OK;
}

// messageCount / entryCount (raft_optimized.go:1014-1048 / 979-1012) over
// [0, l): false where the reference indexes outside the slice (a panic).
template <class R>
__device__ bool count_chain_ok(R& r, u64 base, i64 l, i32 field) {
  i64 i = 0;
  while (i < l) {
    u64 vv[2];
    for (int k = 0; k < 2; ++k) {
      u64 v = 0;
      for (u64 shift = 0;; shift += 7) {
        if (i < 0 || i >= l) return false;
        u8 b = r.at(base + (u64)i);
        i++;
        if (shift < 64) v |= (u64)(b & 0x7F) << shift;
        if (b < 0x80) break;
      }
      vv[k] = v;
      if (k == 0 && (i32)(u32)(v >> 3) != field) return true;
    }
    i = wrap_add(i, (i64)vv[1]);
  }
  return true;
}

// skipRaft (raft.pb.go:5139-5236) on [0, l) relative to base; groups by depth.
template <class R>
__device__ int skip_raft(R& r, u64 base, i64 l, i64& n) {
  i64 i = 0;
  u64 depth = 0;
  for (;;) {
    if (i < 0) return GRW_E_PANIC;  // dAtA[-k] after a wrapped length inside a group
    u64 wire;
    int st = rd_varint(r, base, l, i, wire);
    if (st) return st;
    switch ((int)(wire & 7)) {
      case 0:
        for (u32 shift = 0;; shift += 7) {
          if (shift >= 64) return GRW_E_INT_OVERFLOW;
          if (i >= l) return GRW_E_UNEXPECTED_EOF;
          i++;
          if (r.at(base + (u64)(i - 1)) < 0x80) break;
        }
        break;
      case 1: i = wrap_add(i, 8); break;
      case 2: {
        u64 len;
        if ((st = rd_varint(r, base, l, i, len))) return st;
        i = wrap_add(i, (i64)len);
        if ((i64)len < 0) return GRW_E_INVALID_LENGTH;
        break;
      }
      case 3: depth++; break;
      case 4: depth--; break;
      case 5: i = wrap_add(i, 4); break;
      default: return GRW_E_ILLEGAL_WIRE_TYPE;
    }
    if (depth == 0) {
      n = i;
      return GRW_OK;
    }
  }
}

// ------------------------------------------------------------------ decode --

struct Scratch {
  u64* spans;        // [buf_len/2 + 1] (msg start rel. frame) | (len << 32), slot frame_off/2 + k
  u32* walked;       // [n] messages walked per frame
  u32* first_msg;    // [n]
  u64* walk_err;     // [n] status | level<<8 | panic<<16 | field<<32
  u32* msg_batch;    // [msgs]
  u32* ents_per_msg; // [msgs]
  u32* first_ent;    // [msgs]
  u64* msg_err;      // [msgs] status | level<<8 | field<<32
  u32* ent_pos;      // [msgs] offset of the first Entries field of a canonical message, ~0 = general
  u64* msg_start;    // [msgs] absolute start and length of each message: decode_ents reads
  u32* msg_len;      //        12 B here, not the 120-B record
  u32* first_bad;    // [n] lowest failing message ordinal per frame (atomicMin), ~0 = none
  u32* ent_msg;      // [entries] message whose first entry this is, ~0 for later entries
  // Large frames only (null otherwise): speculative segment chains, see spec_segments.
  u64* stage;        // [buf_len/2 + 2] chain heads of segment g at slot (g << seg_shift)/2 + k
  const struct SegRec* segs;  // [ceil(buf_len/segment)]
  u32 seg_shift;
};

// 1a. Speculative segment walks, launched when frames average >= 4 segments
// of bytes (the transport's large batches, SendQueueLength 8,192 at soft.go:254).
// The walk's fast rule (a Requests field `0a len` with a 1- or 2-byte length)
// is a function of the position alone, so two chains that share one head
// coincide from there on. One wave per segment of the buffer starts
// at the first plausible message head in the segment (`0a len 08`, 08 being
// Message.Type's tag, raft.pb.go Message.MarshalTo) and follows the rule until
// it leaves the segment. walk_frames adopts a segment's chain as soon as its
// own serial walk lands on one of the chain's first kSegProbe heads, and copies
// the staged spans instead of walking them. The chain is frame-agnostic; the
// adopting walk accepts it only when every head and end lies inside its frame.
// Segment size is 1 << seg_shift bytes (kSegShift by default, GRW_SEG_SHIFT in
// the environment overrides it for tuning, 10..16: a head's offset in its
// segment is staged in 16 bits).
constexpr u32 kSegShift = 13;  // A/B on 512 x 8,192 messages: 12..16 -> walk 0.48/0.45/0.52/0.58/0.85 ms
constexpr u32 kSegProbe = 64;
struct SegRec {
  u64 exit;  // absolute: first position >= the segment end, or the head the rule refused
  u32 k;     // chain heads staged (0: no plausible head in the segment)
  u32 pad;
};
// Staged head: head offset in the segment | header bytes << 16 (low word), length (high word).
__device__ __forceinline__ u64 stage_head(u64 s0, u64 st) { return s0 + (st & 0xffff); }

__global__ __launch_bounds__(64) void spec_segments(const u8* buf, u64 buf_len, u64* stage, SegRec* segs, u32 nseg,
                                                    u32 seg_shift) {
  __shared__ uint4 lds_raw[kWin / 16 + 1];
  const u32 g = blockIdx.x;
  if (g >= nseg) return;
  Win w{(u8*)lds_raw, buf, buf_len, 1, 0};
  const u64 s0 = (u64)g << seg_shift;
  const u64 s1 = s0 + (1ull << seg_shift) < buf_len ? s0 + (1ull << seg_shift) : buf_len;
  const u32* d = (const u32*)w.lds;
  // First plausible head, 64 positions per round.
  u64 c = ~0ull;
  for (u64 p = s0; p < s1; p += 64) {
    if (p < w.lo || p >= w.hi || p + 72 > w.lo + kWin) w.load(p);  // uniform; zeros past the buffer
    u32 o = (u32)(p - w.lo) + threadIdx.x;
    u64 pair = (u64)d[o >> 2] | ((u64)d[(o >> 2) + 1] << 32);
    u32 q = (u32)(pair >> (8 * (o & 3)));
    u32 b1 = (q >> 8) & 0xff, b2 = (q >> 16) & 0xff, b3 = q >> 24;
    bool hit = (q & 0xff) == 0x0a && p + threadIdx.x < s1 &&
               ((b1 < 0x80 && b2 == 0x08) || (b1 >= 0x80 && b2 < 0x80 && b3 == 0x08));
    u64 m = __ballot(hit);
    if (m) {
      c = p + (u64)(__ffsll((long long)m) - 1);
      break;
    }
  }
  u32 k = 0;
  u64 i = c;
  if (c != ~0ull) {
    u64* st = stage + (s0 >> 1);
    while (i < s1) {
      u32 q = w.peek4(i);
      if ((q & 0xff) != 0x0a) break;
      u32 b1 = (q >> 8) & 0xff, b2 = (q >> 16) & 0xff;
      u64 len, hdr;
      if (b1 < 0x80) { len = b1; hdr = 2; }
      else if (b2 < 0x80) { len = (b1 & 0x7f) | (b2 << 7); hdr = 3; }
      else break;
      u64 post = i + hdr + len;
      if (post > buf_len) break;
      if (threadIdx.x == 0) st[k] = (u64)((u32)(i - s0) | ((u32)hdr << 16)) | (len << 32);
      k++;
      i = post;
    }
  }
  if (threadIdx.x == 0) segs[g] = SegRec{i, k, 0};
}

__device__ __forceinline__ u64 pack_err(int st, int lvl, int panic, u32 field) {
  return (u64)(u32)st | ((u64)lvl << 8) | ((u64)panic << 16) | ((u64)field << 32);
}

// 1. One wave per frame: the MessageBatch.Unmarshal loop without decoding the
// messages (raft_optimized.go:1050-1202).
template <bool kSpec>
__global__ __launch_bounds__(64) void walk_frames(const u8* buf, u64 buf_len, grw_batch* batches, u32 n,
                                                  Scratch s) {
  __shared__ uint4 lds_raw[kWin / 16 + 1];  // +16 B: peek4 past the window end
  u32 b = blockIdx.x;
  if (b >= n) return;
  Win w{(u8*)lds_raw, buf, buf_len, 1, 0};
  grw_batch bt = batches[b];
  const u64 base = bt.frame_off;
  const i64 l = bt.frame_len;
  u64* spans = s.spans + (base >> 1);
  u64 dep = 0, src_off = 0, binver = 0;
  u32 src_len = 0;
  u32 nm = 0;
  int st = GRW_OK;
  u32 efield = 0;
  i64 first_post = -1;  // post of the first message field: messageCount's start
  i64 i = 0;
  // Segment chain adoption state (large frames, see spec_segments).
  u32 cur_seg = ~0u;
  SegRec rec{0, 0, 0};
  u64 probe = ~0ull;  // this lane's staged head (absolute) in segment cur_seg
  // Fast loop: Requests fields back to back, as MessageBatch.MarshalTo writes
  // them (raft.pb.go:1935-1945), with 1- or 2-byte lengths. It consumes only
  // fields the general loop below would accept unchanged, then hands over.
  while (i + 3 <= l) {
    if (kSpec && nm > 0) {
      const u64 a = base + (u64)i;
      const u32 g = (u32)(a >> s.seg_shift);
      const u64 s0 = (u64)g << s.seg_shift;
      if (g != cur_seg) {
        cur_seg = g;
        rec = s.segs[g];
        u64 st = s.stage[(s0 >> 1) + threadIdx.x];
        probe = threadIdx.x < rec.k && threadIdx.x < kSegProbe ? stage_head(s0, st) : ~0ull;
      }
      const u64 m = __ballot(probe == a);
      // Adopt: heads o..k-1 of the segment's chain are the heads this walk
      // would take from a, provided the chain's end lies inside the frame
      // (then every head h has h + 3 <= l and every end <= l).
      if (m && rec.exit < base + (u64)l) {
        const u32 o = (u32)(__ffsll((long long)m) - 1);
        const u64* st = s.stage + (s0 >> 1) + o;
        const u32 cnt = rec.k - o;
        for (u32 q0 = 0; q0 < cnt; q0 += 8 * 64) {
          u64 v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            u32 t = q0 + (u32)j * 64 + threadIdx.x;
            v[j] = t < cnt ? st[t] : 0;
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            u32 t = q0 + (u32)j * 64 + threadIdx.x;
            if (t < cnt)
              spans[nm + t] = (u64)(u32)(stage_head(s0, v[j]) + ((v[j] >> 16) & 3) - base) |
                              (v[j] & 0xffffffff00000000ull);
          }
        }
        nm += cnt;
        i = (i64)(rec.exit - base);
        continue;
      }
    }
    u32 q = w.peek4(base + (u64)i);
    if ((q & 0xff) != 0x0a) break;
    u32 b1 = (q >> 8) & 0xff, b2 = (q >> 16) & 0xff;
    i64 len, hdr;
    if (b1 < 0x80) { len = b1; hdr = 2; }
    else if (b2 < 0x80) { len = (b1 & 0x7f) | (b2 << 7); hdr = 3; }
    else break;
    i64 post = i + hdr + len;
    if (post > l) break;
    if (nm == 0) first_post = post;
    if (threadIdx.x == 0) spans[nm] = (u64)(u32)(i + hdr) | ((u64)(u32)len << 32);
    nm++;
    i = post;
  }
  while (i < l) {
    i64 pre = i;
    u64 wire;
    if ((st = rd_varint(w, base, l, i, wire))) break;
    i32 field = (i32)(u32)(wire >> 3);
    int wt = (int)(wire & 7);
    if (wt == 4) { st = GRW_E_END_GROUP; break; }
    if (field <= 0) { st = GRW_E_ILLEGAL_TAG; efield = (u32)field; break; }
    if (field == 1 || field == 3) {
      if (wt != 2) { st = GRW_E_WRONG_WIRE_TYPE; efield = (u32)field; break; }
      u64 len;
      if ((st = rd_varint(w, base, l, i, len))) break;
      if ((i64)len < 0) { st = GRW_E_INVALID_LENGTH; break; }
      i64 post = wrap_add(i, (i64)len);
      if (post < 0) { st = GRW_E_PANIC; break; }
      if (post > l) { st = GRW_E_UNEXPECTED_EOF; break; }
      if (field == 1) {
        if (nm == 0) first_post = post;
        if (threadIdx.x == 0) spans[nm] = (u64)(u32)i | ((u64)(u32)(post - i) << 32);
        nm++;
      } else {
        src_off = base + (u64)i;
        src_len = (u32)(post - i);
      }
      i = post;
      continue;
    }
    if (field == 2 || field == 4) {
      if (wt != 0) { st = GRW_E_WRONG_WIRE_TYPE; efield = (u32)field; break; }
      u64 v;
      if ((st = rd_varint(w, base, l, i, v))) break;
      if (field == 2) dep = v; else binver = (u32)v;
      continue;
    }
    i = pre;
    i64 skippy;
    if ((st = skip_raft(w, base + (u64)i, l - i, skippy))) break;
    if (skippy < 0) { st = GRW_E_INVALID_LENGTH; break; }
    if (wrap_add(i, skippy) > l) { st = GRW_E_UNEXPECTED_EOF; break; }
    i += skippy;
  }
  // messageCount ran when the first message was reached. Where the walk went
  // through every field it read the same chain with checked varints, so it
  // cannot have panicked; after a walk error, run it as written.
  int panic = 0;
  if (st != GRW_OK && first_post >= 0) panic = count_chain_ok(w, base + (u64)first_post, l - first_post, 1) ? 0 : 1;
  if (threadIdx.x == 0) {
    s.walked[b] = nm;
    s.walk_err[b] = pack_err(st, GRW_LVL_BATCH, panic, efield);
    batches[b].deployment_id = dep;
    batches[b].source_off = src_off;
    batches[b].source_len = src_len;
    batches[b].bin_ver = (u32)binver;
  }
}

__global__ void map_msgs(const u32* walked, const u32* first_msg, u32 n, u32* msg_batch) {
  u32 b = blockIdx.x;
  if (b >= n) return;
  u32 f = first_msg[b], c = walked[b];
  for (u32 k = threadIdx.x; k < c; k += blockDim.x) msg_batch[f + k] = b;
}

struct MsgOut {
  int st = GRW_OK;
  int lvl = GRW_LVL_MESSAGE;
  u32 field = 0;
};

// Entry.unmarshal (raft_optimized.go:302-650) of [0, l) at absolute `base`.
template <bool kStore>
__device__ __forceinline__ int entry_unmarshal(Rd& r, u64 base, i64 l, grw_entry* o) {
  if (l == 0) return GRW_E_ENTRY_EOF;
  u8 header = r.at(base);
  i64 i = 1;
  u64 term = 0, index = 0, key = 0, client = 0, series = 0, resp = 0;
  i32 type = 0;
#pragma unroll 1
  for (int f = 0; f < 7; ++f) {
    if (f == 2) {  // Type (raft_optimized.go:379-436): u32, no shift cap
      if (header == 2 || header == (2 | 0x80)) {
        if (i + 1 >= l) return GRW_E_ENTRY_EOF;
        u32 x = r.at(base + i);
        i++;
        if (x >= 0x80) {
          x &= 0x7f;
          for (u32 shift = 7;; shift += 7) {
            u32 bb = r.at(base + i);
            i++;
            if (i >= l) return GRW_E_ENTRY_EOF;
            if (bb < 0x80) {
              if (shift < 32) x |= bb << shift;
              break;
            }
            if (shift < 32) x |= (bb & 0x7f) << shift;
          }
        }
        type = (header == 2) ? (i32)x : (i32)(~x + 1);
        header = r.at(base + i);
        i++;
      }
      continue;
    }
    u64 x;
    if (header == (u8)f) {  // varint form, e.g. raft_optimized.go:310-335
      i64 start = i;
      i++;
      if (i >= l) return GRW_E_ENTRY_EOF;
      x = r.at(base + start);
      if (x >= 0x80) {
        x &= 0x7f;
        for (u32 shift = 7;; shift += 7) {
          u64 bb = r.at(base + i);
          i++;
          if (i >= l) return GRW_E_ENTRY_EOF;
          if (bb < 0x80 || shift == 56) {
            x |= bb << shift;
            break;
          }
          x |= (bb & 0x7f) << shift;
        }
      }
    } else if (header == (u8)(f | 0x80)) {  // big-endian fixed form, :336-345
      i64 start = i;
      i += 8;
      if (i >= l) return GRW_E_ENTRY_EOF;
      x = 0;
      for (int k = 0; k < 8; ++k) x = (x << 8) | r.at(base + start + k);
    } else {
      continue;
    }
    switch (f) {
      case 0: term = x; break;
      case 1: index = x; break;
      case 3: key = x; break;
      case 4: client = x; break;
      case 5: series = x; break;
      default: resp = x; break;
    }
    header = r.at(base + i);
    i++;
  }
  u64 cmd_off = 0;
  u32 cmd_len = 0;
  if (header == 7) {  // Cmd, raft_optimized.go:600-637
    if (i >= l) return GRW_E_ENTRY_EOF;
    u64 x = r.at(base + i);
    i++;
    if (x >= 0x80) {
      x &= 0x7f;
      for (u64 shift = 7;; shift += 7) {
        if (i >= l) return GRW_E_ENTRY_EOF;
        u64 bb = r.at(base + i);
        i++;
        if (bb < 0x80) {
          if (shift < 64) x |= bb << shift;
          break;
        }
        if (shift < 64) x |= (bb & 0x7f) << shift;
      }
    }
    if (x > (u64)GRW_COLFER_SIZE_MAX) return GRW_E_ENTRY_MAX;
    i64 start = i;
    i += (i64)x;
    if (i >= l) return i >= (i64)GRW_COLFER_SIZE_MAX ? GRW_E_ENTRY_MAX : GRW_E_ENTRY_EOF;
    cmd_off = base + (u64)start;
    cmd_len = (u32)x;
    header = r.at(base + i);
    i++;
  }
  if (header != 0x7f) return GRW_E_ENTRY_HEADER;
  if (i >= (i64)GRW_COLFER_SIZE_MAX) return GRW_E_ENTRY_MAX;
  if (kStore) {
    o->term = term;
    o->index = index;
    o->key = key;
    o->client_id = client;
    o->series_id = series;
    o->responded_to = resp;
    o->cmd_off = cmd_off;
    o->cmd_len = cmd_len;
    o->type = type;
  }
  return GRW_OK;
}

__device__ __forceinline__ bool zero_snapshot(Rd& r, u64 a, i64 len) {
  if (len == 0) return true;
  if (len != 12) return false;
  for (int k = 0; k < 12; ++k)
    if (r.at(a + k) != kZeroSnap[k]) return false;
  return true;
}

// Message.Unmarshal (raft_optimized.go:653-977) of [0, l) at absolute base.
// kStore = false: fields into m, entries validated and counted (n_ents).
// kStore = true: entries written to ents (the fields pass already succeeded).
template <bool kStore>
__device__ MsgOut message_unmarshal(Rd& r, u64 base, i64 l, grw_message* m, grw_entry* ents, u32& n_ents) {
  MsgOut e;
  i64 i = 0;
  i64 first_ent_post = -1;  // entryCount's start (the first Entries field's post)
  n_ents = 0;
  while (i < l) {
    i64 pre = i;
    u64 wire;
    if ((e.st = rd_varint(r, base, l, i, wire))) break;
    i32 field = (i32)(u32)(wire >> 3);
    int wt = (int)(wire & 7);
    if (wt == 4) { e.st = GRW_E_END_GROUP; break; }
    if (field <= 0) { e.st = GRW_E_ILLEGAL_TAG; e.field = (u32)field; break; }
    if ((field >= 1 && field <= 10) || field == 13) {
      if (wt != 0) { e.st = GRW_E_WRONG_WIRE_TYPE; e.field = (u32)field; break; }
      u64 v;
      if ((e.st = rd_varint(r, base, l, i, v))) break;
      if (!kStore) {
        switch (field) {
          case 1: m->type = (i32)(u32)v; break;
          case 2: m->to = v; break;
          case 3: m->from = v; break;
          case 4: m->cluster_id = v; break;
          case 5: m->term = v; break;
          case 6: m->log_term = v; break;
          case 7: m->log_index = v; break;
          case 8: m->commit = v; break;
          case 9: m->reject = v != 0; break;
          case 10: m->hint = v; break;
          default: m->hint_high = v; break;
        }
      }
      continue;
    }
    if (field == 11 || field == 12) {
      if (wt != 2) { e.st = GRW_E_WRONG_WIRE_TYPE; e.field = (u32)field; break; }
      u64 len;
      if ((e.st = rd_varint(r, base, l, i, len))) break;
      if ((i64)len < 0) { e.st = GRW_E_INVALID_LENGTH; break; }
      i64 post = wrap_add(i, (i64)len);
      if (post < 0) { e.st = GRW_E_PANIC; break; }
      if (post > l) { e.st = GRW_E_UNEXPECTED_EOF; break; }
      if (field == 11) {
        if (first_ent_post < 0) first_ent_post = post;
        int st = entry_unmarshal<kStore>(r, base + (u64)i, post - i, kStore ? ents + n_ents : nullptr);
        if (st) { e.st = st; e.lvl = GRW_LVL_ENTRY; break; }
        n_ents++;
      } else if (!kStore) {
        if (!zero_snapshot(r, base + (u64)i, post - i)) m->snapshot_host = 1;
        m->snapshot_off = base + (u64)i;
        m->snapshot_len = (u32)(post - i);
      }
      i = post;
      continue;
    }
    i = pre;
    i64 skippy;
    if ((e.st = skip_raft(r, base + (u64)i, l - i, skippy))) break;
    if (skippy < 0) { e.st = GRW_E_INVALID_LENGTH; break; }
    if (wrap_add(i, skippy) > l) { e.st = GRW_E_UNEXPECTED_EOF; break; }
    i += skippy;
  }
  // entryCount ran at the first Entries field; only a later error can hide a
  // chain that runs off the message (see walk_frames).
  if (e.st != GRW_OK && first_ent_post >= 0 &&
      !count_chain_ok(r, base + (u64)first_ent_post, l - first_ent_post, 11)) {
    e.st = GRW_E_PANIC;
    e.lvl = GRW_LVL_MESSAGE;
    e.field = 0;
  }
  return e;
}

// Varint that only succeeds where rd_varint would (no error paths to report).
__device__ __forceinline__ bool fast_varint(Rd& r, u64 base, i64 l, i64& i, u64& v) {
  v = 0;
#pragma unroll 1
  for (u32 shift = 0; shift < 64; shift += 7) {
    if (i >= l) return false;
    u8 b = r.at(base + (u64)i);
    i++;
    v |= (u64)(b & 0x7F) << shift;
    if (b < 0x80) return true;
  }
  return false;
}

struct Fast {
  u64 f[11];  // Type To From ClusterId Term LogTerm LogIndex Commit Reject Hint HintHigh
  u64 snap_off;
  u32 snap_len, n_ents, ent_pos;
  u8 snap_host;
};

// The canonical layout Message.MarshalTo writes (raft.pb.go:1747-1809): fields
// 1..10 in order, Entries, Snapshot, HintHigh, nothing else. Returns true only
// for such a message whose entries are all valid, with the values the general
// decoder would produce; anything else goes to message_unmarshal.
__device__ __forceinline__ bool fast_message(Rd& r, u64 base, i64 l, Fast& o) {
  i64 i = 0;
#pragma unroll
  for (int k = 0; k < 10; ++k) {  // unrolled: o.f[k] stays in registers
    if (i >= l || r.at(base + (u64)i) != (u8)((k + 1) << 3)) return false;
    i++;
    if (!fast_varint(r, base, l, i, o.f[k])) return false;
  }
  o.n_ents = 0;
  o.ent_pos = (u32)i;
  while (i < l && r.at(base + (u64)i) == 0x5a) {
    i++;
    u64 len;
    if (!fast_varint(r, base, l, i, len) || len > (u64)l) return false;
    i64 post = i + (i64)len;
    if (post > l) return false;
    if (entry_unmarshal<false>(r, base + (u64)i, post - i, nullptr)) return false;
    o.n_ents++;
    i = post;
  }
  if (i >= l || r.at(base + (u64)i) != 0x62) return false;
  i++;
  u64 len;
  if (!fast_varint(r, base, l, i, len) || len > (u64)l) return false;
  i64 post = i + (i64)len;
  if (post > l) return false;
  o.snap_off = base + (u64)i;
  o.snap_len = (u32)len;
  o.snap_host = zero_snapshot(r, base + (u64)i, (i64)len) ? 0 : 1;
  i = post;
  if (i >= l || r.at(base + (u64)i) != 0x68) return false;
  i++;
  if (!fast_varint(r, base, l, i, o.f[10])) return false;
  return i == l;
}

// The general decoder, kept out of line: only non-canonical or failing
// messages take it.
__device__ __noinline__ MsgOut general_message(const u8* buf, u64 buf_len, u64 base, i64 l, grw_message* m,
                                               u32* ne) {
  Rd r(buf, buf_len);
  return message_unmarshal<false>(r, base, l, m, nullptr, *ne);
}

__device__ __noinline__ void general_entries(const u8* buf, u64 buf_len, u64 base, i64 l, grw_entry* ents) {
  Rd r(buf, buf_len);
  u32 ne;
  message_unmarshal<true>(r, base, l, nullptr, ents, ne);
}

// Stage the bytes a block's messages cover, [lo, hi) capped at kStage, into
// LDS with coalesced 16-B loads; lanes then read their messages from LDS
// (Rd falls back to global loads outside the window).
constexpr int kStage = 16384;
__device__ __forceinline__ void stage_block(Rd& r, uint4* lds, u64 lo, u64 hi, bool active) {
  __shared__ unsigned long long s_lo, s_hi;
  if (threadIdx.x == 0) { s_lo = ~0ull; s_hi = 0; }
  __syncthreads();
  if (active) {
    atomicMin(&s_lo, (unsigned long long)lo);
    atomicMax(&s_hi, (unsigned long long)hi);
  }
  __syncthreads();
  u64 a = s_lo & ~15ull, b = s_hi;
  u64 cap_end = r.len & ~15ull;  // whole chunks inside the buffer only
  if (b > a + kStage) b = a + kStage;
  if (b > cap_end) b = cap_end;
  b &= ~15ull;
  if ((((uintptr_t)r.buf) & 15) != 0 || s_lo == ~0ull || b <= a) { a = b = 0; }
  for (u64 k = threadIdx.x; k < (b - a) >> 4; k += blockDim.x) lds[k] = *(const uint4*)(r.buf + a + (k << 4));
  __syncthreads();
  r.lds = lds;
  r.llo = a;
  r.lhi = b;
}

__global__ __launch_bounds__(256) void decode_msgs(const u8* buf, u64 buf_len, const grw_batch* batches, u32 total,
                                                   Scratch s, grw_message* msgs) {
  __shared__ uint4 lds[kStage / 16];
  u32 j = blockIdx.x * blockDim.x + threadIdx.x;
  bool act = j < total;
  u64 start = 0;
  u32 len = 0, b = 0;
  if (act) {
    b = s.msg_batch[j];
    u32 k = j - s.first_msg[b];
    u64 fo = batches[b].frame_off;
    u64 sp = s.spans[(fo >> 1) + k];
    start = fo + (u32)sp;
    len = (u32)(sp >> 32);
  }
  Rd r(buf, buf_len);
  stage_block(r, lds, start, start + len, act);
  if (!act) return;
  grw_message* mo = msgs + j;
  Fast f;
  if (fast_message(r, start, len, f)) {
    mo->type = (i32)(u32)f.f[0];
    mo->to = f.f[1];
    mo->from = f.f[2];
    mo->cluster_id = f.f[3];
    mo->term = f.f[4];
    mo->log_term = f.f[5];
    mo->log_index = f.f[6];
    mo->commit = f.f[7];
    mo->reject = f.f[8] != 0;
    mo->hint = f.f[9];
    mo->hint_high = f.f[10];
    mo->snapshot_off = f.snap_off;
    mo->snapshot_len = f.snap_len;
    mo->snapshot_host = f.snap_host;
    mo->msg_off = start;
    mo->msg_len = len;
    mo->batch = b;
    mo->n_entries = f.n_ents;
    s.ents_per_msg[j] = f.n_ents;
    s.ent_pos[j] = f.ent_pos;
    s.msg_start[j] = start;
    s.msg_len[j] = len;
    s.msg_err[j] = 0;
    return;
  }
  grw_message m;
  memset(&m, 0, sizeof(m));
  u32 ne = 0;
  MsgOut e = general_message(buf, buf_len, start, len, &m, &ne);
  m.msg_off = start;
  m.msg_len = len;
  m.batch = b;
  m.n_entries = ne;
  *mo = m;
  s.ents_per_msg[j] = e.st ? 0 : ne;
  s.ent_pos[j] = 0xFFFFFFFFu;
  s.msg_start[j] = start;
    s.msg_len[j] = len;
  s.msg_err[j] = pack_err(e.st, e.lvl, 0, e.field);
  if (e.st) atomicMin(&s.first_bad[b], j - s.first_msg[b]);
}

// 5a. One lane per message: first_entry into the record, and the entry ->
// message map decode_ents runs over (messages without entries get no lane).
__global__ void map_ents(u32 total, Scratch s, grw_message* msgs) {
  u32 j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= total) return;
  u32 fe = s.first_ent[j];
  msgs[j].first_entry = fe;
  if (s.ents_per_msg[j]) s.ent_msg[fe] = j;
}

// 5b. One lane per entry; the lane of a message's first entry decodes all of
// that message's entries, so a wave holds only messages that carry entries.
// No LDS staging: with a lane per entry the block's messages are spread over
// 4x more bytes than its entries (A/B: staged 0.377 vs unstaged 0.359 ms).
__global__ __launch_bounds__(64) void decode_ents(const u8* buf, u64 buf_len, u32 tents, Scratch s,
                                                  grw_entry* ents) {
  u32 e = blockIdx.x * blockDim.x + threadIdx.x;
  u32 j = e < tents ? s.ent_msg[e] : ~0u;
  bool act = j != ~0u;
  u32 n = 0, l = 0, pos = 0, fe = e;
  u64 base = 0;
  if (act) {
    n = s.ents_per_msg[j];
    base = s.msg_start[j];
    l = s.msg_len[j];
    pos = s.ent_pos[j];
  }
  Rd r(buf, buf_len);
  if (!act) return;
  if (pos == 0xFFFFFFFFu) {
    general_entries(buf, buf_len, base, l, ents + fe);
    return;
  }
  // Canonical message: its n Entries fields start at pos, back to back.
  i64 i = pos;
  for (u32 k = 0; k < n; ++k) {
    i++;  // 0x5a
    u64 len;
    fast_varint(r, base, l, i, len);
    entry_unmarshal<true>(r, base + (u64)i, (i64)len, ents + fe + k);
    i += (i64)len;
  }
}

// 6. Status = the first error in wire order: a messageCount panic (raised at
// the first message), else the first failing message, else the walk's error.
__global__ void finish_frames(grw_batch* batches, u32 n, Scratch s) {
  u32 b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  u64 we = s.walk_err[b];
  u32 f = s.first_msg[b], c = s.walked[b];
  grw_batch& bt = batches[b];
  bt.first_msg = f;
  int st = (int)(we & 0xff), lvl = (int)((we >> 8) & 0xff);
  u32 field = (u32)(we >> 32), at = c;
  if ((we >> 16) & 1) {
    st = GRW_E_PANIC; lvl = GRW_LVL_BATCH; field = 0; at = 0;
  } else if (s.first_bad[b] < c) {  // the first failing message, found by decode_msgs' atomicMin
    const u32 k = s.first_bad[b];
    const u64 me = s.msg_err[f + k];
    st = (int)(me & 0xff); lvl = (int)((me >> 8) & 0xff); field = (u32)(me >> 32); at = k;
  }
  bt.status = st;
  bt.err_level = (u8)(st ? lvl : GRW_LVL_BATCH);
  bt.err_field = st ? field : 0;
  bt.err_msg = st ? at : 0;
  bt.n_msgs = st ? at : c;
}

// ------------------------------------------------------------------ encode --

// Varint length of x, branch-free: ceil(bits / 7) with bits(0) taken as 1.
__device__ __forceinline__ int sov(u64 x) { return (70 - __clzll((long long)(x | 1))) / 7; }

// Entry.Size (raft_optimized.go:78-153); -1 where it panics.
__device__ i64 entry_size(const grw_entry& o) {
  i64 l = 1;
  const u64 f64[6] = {o.term, o.index, o.key, o.client_id, o.series_id, o.responded_to};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    u64 x = f64[k];
    if (x >= (1ull << 49)) l += 9;
    else if (x != 0) l += 1 + sov(x);
    if (k == 1 && o.type != 0) {
      u32 x32 = (u32)o.type;
      if (o.type < 0) x32 = ~x32 + 1;
      l += 1 + sov(x32);
    }
  }
  if (u64 x = o.cmd_len) {
    if (x > GRW_COLFER_SIZE_MAX) return -1;
    l += (i64)x + 1 + sov(x);
  }
  if (l > (i64)GRW_COLFER_SIZE_MAX) return -1;
  return l;
}

__device__ __forceinline__ u64 snap_size(const grw_message& m) { return m.snapshot_len ? m.snapshot_len : 12; }

// Message.Size (raft.pb.go:2219-2245); -1 where an entry's Size panics.
__device__ i64 message_size(const grw_message& m, const grw_entry* ents) {
  i64 n = 1 + sov((u64)(i64)m.type);
  n += 7 + sov(m.to) + sov(m.from) + sov(m.cluster_id) + sov(m.term) + sov(m.log_term) + sov(m.log_index) +
       sov(m.commit);
  n += 2 + 1 + sov(m.hint);
  for (u32 k = 0; k < m.n_entries; ++k) {
    i64 l = entry_size(ents[m.first_entry + k]);
    if (l < 0) return -1;
    n += 1 + l + sov((u64)l);
  }
  u64 sl = snap_size(m);
  n += 1 + (i64)sl + sov(sl) + 1 + sov(m.hint_high);
  return n;
}

// Byte writer over out[lo, hi): dword stores for the dwords it owns whole,
// byte stores at the two ends it may share with a neighbouring record.
// Alignment is taken from the address, so any output pointer works.
struct Wr {
  u8* p;       // next byte
  u8* lo;
  u8* hi;
  u32 acc;     // bytes of the dword being assembled
  __device__ Wr(u8* out, u64 start, u64 end) : p(out + start), lo(out + start), hi(out + end), acc(0) {}
  __device__ __forceinline__ void put(u8 v) {
    uintptr_t a = (uintptr_t)p;
    acc |= (u32)v << (8 * (a & 3));
    p++;
    if ((((uintptr_t)p) & 3) == 0 || p == hi) flush((u8*)(a & ~(uintptr_t)3));
  }
  __device__ __forceinline__ void flush(u8* d) {
    if (d >= lo && d + 4 <= hi) {
      *(u32*)d = acc;
    } else {
      for (u8* q = (d > lo ? d : lo); q < d + 4 && q < hi; ++q) *q = (u8)(acc >> (8 * (q - d)));
    }
    acc = 0;
  }
  __device__ __forceinline__ void varint(u64 v) {
    while (v >= 0x80) { put((u8)(v | 0x80)); v >>= 7; }
    put((u8)v);
  }
};

__device__ void entry_write(Wr& w, const grw_entry& o, const u8* payload) {
  const u64 f64[6] = {o.term, o.index, o.key, o.client_id, o.series_id, o.responded_to};
  const u8 hdr[6] = {0, 1, 3, 4, 5, 6};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    u64 x = f64[k];
    if (x >= (1ull << 49)) {
      w.put(hdr[k] | 0x80);
      for (int s = 0; s < 8; ++s) w.put((u8)(x >> (56 - 8 * s)));
    } else if (x != 0) {
      w.put(hdr[k]);
      w.varint(x);
    }
    if (k == 1 && o.type != 0) {
      u32 x32 = (u32)o.type;
      if (o.type >= 0) w.put(2);
      else { x32 = ~x32 + 1; w.put(2 | 0x80); }
      w.varint(x32);
    }
  }
  if (o.cmd_len) {
    w.put(7);
    w.varint(o.cmd_len);
    const u8* p = payload + o.cmd_off;
    for (u32 k = 0; k < o.cmd_len; ++k) w.put(p[k]);
  }
  w.put(0x7f);
}

struct EncScratch {
  u64* fsz;        // [msgs] size of the message's field in the batch (0 if it panics)
  u64* pos;        // [msgs+1] exclusive scan of fsz
  u64* flen;       // [n] frame lengths
  u64* foff;       // [n] frame offsets
  u32* msg_batch;  // [msgs]
  u32* bad;        // [1] batches not contiguous in message order
};

__global__ void size_msgs(const grw_message* msgs, u32 total, const grw_entry* ents, EncScratch s, u32* panic_flag) {
  u32 j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= total) return;
  i64 l = message_size(msgs[j], ents);
  if (l < 0) {
    s.fsz[j] = 0;
    atomicOr(&panic_flag[s.msg_batch[j]], 1u);
  } else {
    s.fsz[j] = 1 + (u64)l + (u64)sov((u64)l);
  }
}

__global__ void enc_map(const grw_batch* batches, u32 n, u32 total, EncScratch s, u32* panic_flag) {
  u32 b = blockIdx.x;
  if (b >= n) return;
  u32 f = batches[b].first_msg, c = batches[b].n_msgs;
  if (threadIdx.x == 0) panic_flag[b] = 0;
  for (u32 k = threadIdx.x; k < c; k += blockDim.x)
    if (f + k < total) s.msg_batch[f + k] = b;
}

__global__ void check_contig(const grw_batch* batches, u32 n, u32 total, EncScratch s) {
  u32 b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  u32 f = batches[b].first_msg, c = batches[b].n_msgs;
  u32 expect_next = (b + 1 < n) ? batches[b + 1].first_msg : total;
  if ((u64)f + c > total || (b + 1 < n && f + c != expect_next) || (b == 0 && f != 0) ||
      (b + 1 == n && f + c != total))
    atomicOr(s.bad, 1u);
}

__global__ void frame_sizes(grw_batch* batches, u32 n, EncScratch s, const u32* panic_flag) {
  u32 b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const grw_batch& bt = batches[b];
  u64 body = s.pos[bt.first_msg + bt.n_msgs] - s.pos[bt.first_msg];
  u64 tail = 1 + sov(bt.deployment_id) + 1 + (u64)bt.source_len + sov(bt.source_len) + 1 + sov(bt.bin_ver);
  s.flen[b] = panic_flag[b] ? 0 : body + tail;
  if (!panic_flag[b] && body + tail > 0xFFFFFFFFull) atomicOr(s.bad, 2u);  // frame_len is 32-bit
}

// Every record an encode reads must lie inside the arrays it was given: a
// message's entries inside ents, every Cmd / Snapshot / SourceAddress inside the
// payload buffer. One bad record fails the call (GR_EINVAL) before any byte is
// read out of range.
__device__ __forceinline__ bool out_of(u64 off, u64 len, u64 cap) { return len && (off > cap || len > cap - off); }
__global__ void check_records(const grw_batch* batches, u32 n, const grw_message* msgs, u32 nm, const grw_entry* ents,
                              u64 n_ents, u64 payload_len, EncScratch s) {
  const u64 t = blockIdx.x * (u64)blockDim.x + threadIdx.x;
  bool bad = false;
  if (t < nm) {
    const grw_message& m = msgs[t];
    bad |= (u64)m.first_entry + m.n_entries > n_ents;
    bad |= out_of(m.snapshot_off, m.snapshot_len, payload_len);
  }
  if (t < n_ents) bad |= out_of(ents[t].cmd_off, ents[t].cmd_len, payload_len);
  if (t < n) bad |= out_of(batches[t].source_off, batches[t].source_len, payload_len);
  if (bad) atomicOr(s.bad, 1u);
}

__global__ void frame_finish(grw_batch* batches, u32 n, EncScratch s, const u32* panic_flag) {
  u32 b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  batches[b].frame_off = s.foff[b];
  batches[b].frame_len = (u32)s.flen[b];
  batches[b].status = panic_flag[b] ? GRW_E_PANIC : GRW_OK;
}

__device__ __forceinline__ void write_msg(u32 j, u64 at, const grw_message* msgs, const grw_entry* ents,
                                          const u8* payload, EncScratch s, u8* out) {
  const grw_message m = msgs[j];
  // fsz = 1 + l + sov(l) with l = Message.Size(); l + sov(l) rises strictly
  // with l, so l is found from fsz in a few steps instead of re-reading the
  // entries (the batch did not panic, so size_msgs stored a real size).
  const u64 fsz = s.fsz[j];
  u64 l = fsz - 2;
  while (1 + l + (u64)sov(l) != fsz) --l;
  Wr w(out, at, at + fsz);
  w.put(0x0a);
  w.varint(l);
  w.put(0x08); w.varint((u64)(i64)m.type);
  w.put(0x10); w.varint(m.to);
  w.put(0x18); w.varint(m.from);
  w.put(0x20); w.varint(m.cluster_id);
  w.put(0x28); w.varint(m.term);
  w.put(0x30); w.varint(m.log_term);
  w.put(0x38); w.varint(m.log_index);
  w.put(0x40); w.varint(m.commit);
  w.put(0x48); w.put(m.reject ? 1 : 0);
  w.put(0x50); w.varint(m.hint);
  for (u32 k = 0; k < m.n_entries; ++k) {
    const grw_entry e = ents[m.first_entry + k];
    w.put(0x5a);
    w.varint((u64)entry_size(e));
    entry_write(w, e, payload);
  }
  w.put(0x62);
  w.varint(snap_size(m));
  if (m.snapshot_len) {
    const u8* p = payload + m.snapshot_off;
    for (u32 k = 0; k < m.snapshot_len; ++k) w.put(p[k]);
  } else {
    for (int k = 0; k < 12; ++k) w.put(kZeroSnap[k]);
  }
  w.put(0x68); w.varint(m.hint_high);
}

// One lane per message. A block whose messages span at most kOutStage bytes
// (and whose batches did not panic) assembles them in LDS and stores the span
// with coalesced 16-B writes; bytes between frames (tails) are written by
// write_tails afterwards. Writing the records straight to HBM, each wave's
// dword stores touched ~60 lines at once and partial lines were evicted:
// WRITE_SIZE was ~5x the output (profiles/r01_wire_h/pmc).
constexpr u32 kOutStage = 24576;
__global__ __launch_bounds__(256) void write_msgs(const grw_batch* batches, const grw_message* msgs, u32 total,
                                                  const grw_entry* ents, const u8* payload, EncScratch s,
                                                  const u32* panic_flag, u8* out) {
  __shared__ uint4 img[kOutStage / 16];
  __shared__ unsigned long long s_lo, s_hi;
  __shared__ int s_bad;
  u32 j = blockIdx.x * blockDim.x + threadIdx.x;
  bool act = j < total;
  u32 b = 0;
  bool bad = false;
  u64 at = 0, end = 0;
  if (threadIdx.x == 0) { s_lo = ~0ull; s_hi = 0; s_bad = 0; }
  __syncthreads();
  if (act) {
    b = s.msg_batch[j];
    bad = panic_flag[b] != 0;
    at = s.foff[b] + (s.pos[j] - s.pos[batches[b].first_msg]);
    end = at + s.fsz[j];
    if (bad) atomicOr(&s_bad, 1);
    else {
      atomicMin(&s_lo, (unsigned long long)at);
      atomicMax(&s_hi, (unsigned long long)end);
    }
  }
  __syncthreads();
  const u64 lo = s_lo, hi = s_hi, alo = lo & ~15ull;
  const bool staged = s_bad == 0 && hi > lo && hi - alo <= kOutStage;
  if (!staged) {
    if (act && !bad) write_msg(j, at, msgs, ents, payload, s, out);
    return;
  }
  if (act) write_msg(j, at - alo, msgs, ents, payload, s, (u8*)img);
  __syncthreads();
  for (u64 off = (u64)threadIdx.x * 16; alo + off < hi; off += (u64)blockDim.x * 16) {
    const u64 g = alo + off;
    const uint4 v = img[off >> 4];
    u8* q = out + g;
    if (g >= lo && g + 16 <= hi && (((uintptr_t)q) & 15) == 0) {
      *(uint4*)q = v;
    } else {
      const u8* vb = (const u8*)&v;
      for (int k = 0; k < 16; ++k)
        if (g + k >= lo && g + k < hi) q[k] = vb[k];
    }
  }
}

__global__ void write_tails(const grw_batch* batches, u32 n, const u8* payload, EncScratch s, const u32* panic_flag,
                            u8* out) {
  u32 b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n || panic_flag[b]) return;
  const grw_batch& bt = batches[b];
  u64 end = s.foff[b] + s.flen[b];
  u64 tail = 1 + sov(bt.deployment_id) + 1 + (u64)bt.source_len + sov(bt.source_len) + 1 + sov(bt.bin_ver);
  Wr w(out, end - tail, end);
  w.put(0x10); w.varint(bt.deployment_id);
  w.put(0x1a); w.varint(bt.source_len);
  const u8* p = payload + bt.source_off;
  for (u32 k = 0; k < bt.source_len; ++k) w.put(p[k]);
  w.put(0x20); w.varint(bt.bin_ver);
}

}  // namespace grw

// ------------------------------------------------------------------- C-ABI --

using namespace grw;

struct grw_ctx {
  struct Buf {
    void* p = nullptr;
    size_t n = 0;
  };
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[6] = {};
  grw_timing timing{};
  Buf spans, walked, first_msg, walk_err, msg_batch, ents_per_msg, first_ent, msg_err, ent_pos, msg_start, msg_len, first_bad, tmp, scal;
  Buf ent_msg;
  Buf stage, segs;  // large-frame segment chains (spec_segments)
  Buf fsz, pos, flen, foff, pflag;
  // host-path staging
  Buf d_buf, d_batches, d_msgs, d_ents;
  u8* h_scal = nullptr;
  std::recursive_mutex mu;  // host and device entry points alike: one call at a time per context
};

#define HIPCHK(x)                            \
  do {                                       \
    hipError_t _e = (x);                     \
    if (_e != hipSuccess) return GR_EDEVICE; \
  } while (0)

static int grow(grw_ctx::Buf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.n >= bytes) return GR_OK;
  if (b.p) hipFree(b.p);
  b.p = nullptr;
  b.n = 0;
  size_t want = bytes + bytes / 4;
  if (hipMalloc(&b.p, want) != hipSuccess) return GR_ENOMEM;
  b.n = want;
  return GR_OK;
}

template <class T>
static int scan_excl(grw_ctx* c, const T* in, T* out, size_t n) {
  if (n == 0) return GR_OK;
  if (n >= 0xFFFFFFFFull) return GR_EINVAL;
  if (int r = grow(c->tmp, (size_t)gr::scan::scan_tiles_of(n) * sizeof(T))) return r;
  HIPCHK(gr::scan::exclusive_scan<T>(in, out, (uint32_t)n, (T*)c->tmp.p, c->stream));
  return GR_OK;
}

static inline unsigned nblk(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

extern "C" {

int grw_create(uint32_t device, grw_ctx** out) {
  if (!out) return GR_EINVAL;
  *out = nullptr;
  int cnt = 0;
  if (hipGetDeviceCount(&cnt) != hipSuccess || (int)device >= cnt) return GR_EDEVICE;
  grw_ctx* c = new (std::nothrow) grw_ctx();
  if (!c) return GR_ENOMEM;
  c->device = (int)device;
  if (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return GR_EDEVICE;
  }
  for (auto& e : c->ev) hipEventCreate(&e);
  if (hipHostMalloc((void**)&c->h_scal, 64) != hipSuccess) {
    delete c;
    return GR_ENOMEM;
  }
  *out = c;
  return GR_OK;
}

void grw_destroy(grw_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  grw_ctx::Buf* bufs[] = {&c->spans, &c->walked, &c->first_msg, &c->walk_err, &c->msg_batch, &c->ents_per_msg,
                          &c->first_ent, &c->msg_err, &c->ent_pos, &c->msg_start, &c->msg_len, &c->first_bad, &c->ent_msg, &c->stage, &c->segs, &c->tmp, &c->scal, &c->fsz, &c->pos, &c->flen, &c->foff,
                          &c->pflag, &c->d_buf, &c->d_batches, &c->d_msgs, &c->d_ents};
  for (auto* b : bufs)
    if (b->p) hipFree(b->p);
  for (auto& e : c->ev)
    if (e) hipEventDestroy(e);
  if (c->h_scal) hipHostFree(c->h_scal);
  hipStreamDestroy(c->stream);
  delete c;
}

const char* grw_status_name(int s) {
  static const char* names[] = {"ok", "ErrIntOverflowRaft", "io.ErrUnexpectedEOF", "ErrInvalidLengthRaft",
                                "wiretype end group for non-group", "illegal tag", "wrong wireType",
                                "illegal wireType", "colfer io.EOF", "ColferError", "ColferMax", "panic"};
  return (s >= 0 && s <= GRW_E_PANIC) ? names[s] : "unknown";
}

int grw_decode_device(grw_ctx* c, const uint8_t* d_buf, size_t buf_len, grw_batch* d_batches, size_t n,
                      grw_message* d_msgs, size_t msg_cap, grw_entry* d_ents, size_t ent_cap, size_t* n_msgs,
                      size_t* n_ents) {
  if (!c || !n_msgs || !n_ents || (n && (!d_buf || !d_batches)) || n > 0xFFFFFFFFull) return GR_EINVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);  // shares scratch, stream and events with every other call
  *n_msgs = *n_ents = 0;
  if (n == 0) return GR_OK;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  int r;
  if ((r = grow(c->spans, (buf_len / 2 + 2) * 8)) || (r = grow(c->walked, n * 4)) || (r = grow(c->first_msg, n * 4)) ||
      (r = grow(c->walk_err, n * 8)) || (r = grow(c->scal, 64)) || (r = grow(c->first_bad, n * 4)))
    return r;
  Scratch sc{};
  sc.spans = (u64*)c->spans.p;
  sc.walked = (u32*)c->walked.p;
  sc.first_msg = (u32*)c->first_msg.p;
  sc.walk_err = (u64*)c->walk_err.p;
  sc.first_bad = (u32*)c->first_bad.p;
  HIPCHK(hipMemsetAsync(sc.first_bad, 0xFF, n * 4, s));
  u32 seg_shift = kSegShift;
  if (const char* e = getenv("GRW_SEG_SHIFT")) {
    int v = atoi(e);
    if (v >= 10 && v <= 16) seg_shift = (u32)v;
  }
  const bool spec = buf_len / n >= (4ull << seg_shift);  // >= 4 segments per frame on average
  const u64 nseg = (buf_len + (1ull << seg_shift) - 1) >> seg_shift;
  sc.seg_shift = seg_shift;
  if (spec) {
    if ((r = grow(c->stage, (buf_len / 2 + 2 + kSegProbe) * 8)) || (r = grow(c->segs, nseg * sizeof(SegRec)))) return r;
    sc.stage = (u64*)c->stage.p;
    sc.segs = (const SegRec*)c->segs.p;
  }
  HIPCHK(hipEventRecord(c->ev[0], s));
  if (spec) {
    spec_segments<<<(unsigned)nseg, 64, 0, s>>>(d_buf, buf_len, sc.stage, (SegRec*)c->segs.p, (u32)nseg, seg_shift);
    HIPCHK(hipGetLastError());
  }
  if (spec)
    walk_frames<true><<<(unsigned)n, 64, 0, s>>>(d_buf, buf_len, d_batches, (u32)n, sc);
  else
    walk_frames<false><<<(unsigned)n, 64, 0, s>>>(d_buf, buf_len, d_batches, (u32)n, sc);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev[1], s));
  if ((r = scan_excl<u32>(c, sc.walked, sc.first_msg, n))) return r;
  // total = first_msg[n-1] + walked[n-1]
  HIPCHK(hipMemcpyAsync(c->h_scal, sc.first_msg + n - 1, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(c->h_scal + 4, sc.walked + n - 1, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  u32 total = ((u32*)c->h_scal)[0] + ((u32*)c->h_scal)[1];
  if ((r = grow(c->msg_batch, (size_t)total * 4 + 4)) || (r = grow(c->ents_per_msg, (size_t)total * 4 + 4)) ||
      (r = grow(c->first_ent, (size_t)total * 4 + 4)) || (r = grow(c->msg_err, (size_t)total * 8 + 8)) ||
      (r = grow(c->ent_pos, (size_t)total * 4 + 4)) || (r = grow(c->msg_start, (size_t)total * 8 + 8)) ||
      (r = grow(c->msg_len, (size_t)total * 4 + 4)))
    return r;
  sc.ent_pos = (u32*)c->ent_pos.p;
  sc.msg_start = (u64*)c->msg_start.p;
  sc.msg_len = (u32*)c->msg_len.p;
  sc.msg_batch = (u32*)c->msg_batch.p;
  sc.ents_per_msg = (u32*)c->ents_per_msg.p;
  sc.first_ent = (u32*)c->first_ent.p;
  sc.msg_err = (u64*)c->msg_err.p;
  if (total > msg_cap || (total && !d_msgs)) {
    *n_msgs = total;
    return GR_ECAPACITY;
  }
  if (total) {
    map_msgs<<<(unsigned)n, 64, 0, s>>>(sc.walked, sc.first_msg, (u32)n, sc.msg_batch);
    HIPCHK(hipEventRecord(c->ev[2], s));
    decode_msgs<<<nblk(total, 256), 256, 0, s>>>(d_buf, buf_len, d_batches, total, sc, d_msgs);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev[3], s));
    if ((r = scan_excl<u32>(c, sc.ents_per_msg, sc.first_ent, total))) return r;
    HIPCHK(hipMemcpyAsync(c->h_scal, sc.first_ent + total - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(c->h_scal + 4, sc.ents_per_msg + total - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  } else {
    HIPCHK(hipEventRecord(c->ev[2], s));
    HIPCHK(hipEventRecord(c->ev[3], s));
    memset(c->h_scal, 0, 8);
  }
  u32 tents = ((u32*)c->h_scal)[0] + ((u32*)c->h_scal)[1];
  *n_msgs = total;
  *n_ents = tents;
  if (tents > ent_cap || (tents && !d_ents)) return GR_ECAPACITY;
  if (tents && (r = grow(c->ent_msg, (size_t)tents * 4))) return r;
  sc.ent_msg = (u32*)c->ent_msg.p;
  HIPCHK(hipEventRecord(c->ev[4], s));
  if (total) {
    if (tents) HIPCHK(hipMemsetAsync(sc.ent_msg, 0xFF, (size_t)tents * 4, s));
    map_ents<<<nblk(total, 256), 256, 0, s>>>(total, sc, d_msgs);
    HIPCHK(hipGetLastError());
    if (tents) {
      decode_ents<<<nblk(tents, 64), 64, 0, s>>>(d_buf, buf_len, tents, sc, d_ents);
      HIPCHK(hipGetLastError());
    }
  }
  finish_frames<<<nblk(n, 256), 256, 0, s>>>(d_batches, (u32)n, sc);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev[5], s));
  HIPCHK(hipStreamSynchronize(s));
  float t01 = 0, t12 = 0, t23 = 0, t45 = 0, t05 = 0;
  hipEventElapsedTime(&t01, c->ev[0], c->ev[1]);
  hipEventElapsedTime(&t12, c->ev[1], c->ev[2]);
  hipEventElapsedTime(&t23, c->ev[2], c->ev[3]);
  hipEventElapsedTime(&t45, c->ev[4], c->ev[5]);
  hipEventElapsedTime(&t05, c->ev[0], c->ev[5]);
  c->timing = grw_timing{t01, t12, t23, t45, t05};
  return GR_OK;
}

int grw_decode(grw_ctx* c, const uint8_t* buf, size_t buf_len, grw_batch* batches, size_t n, grw_message* msgs,
               size_t msg_cap, grw_entry* ents, size_t ent_cap, size_t* n_msgs, size_t* n_ents) {
  if (!c || !n_msgs || !n_ents || (n && (!buf || !batches))) return GR_EINVAL;
  for (size_t b = 0; b < n; ++b)  // in range, written so that it cannot wrap
    if (batches[b].frame_off > buf_len || batches[b].frame_len > buf_len - batches[b].frame_off) return GR_EINVAL;
  if (n > 1) {  // frames must not overlap (their spans share scratch slots)
    std::vector<std::pair<u64, u64>> iv(n);
    for (size_t b = 0; b < n; ++b) iv[b] = {batches[b].frame_off, batches[b].frame_off + batches[b].frame_len};
    std::sort(iv.begin(), iv.end());
    for (size_t b = 1; b < n; ++b)
      if (iv[b].first < iv[b - 1].second) return GR_EINVAL;
  }
  std::lock_guard<std::recursive_mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  int r;
  if ((r = grow(c->d_buf, buf_len + 16)) || (r = grow(c->d_batches, n * sizeof(grw_batch)))) return r;
  HIPCHK(hipMemcpyAsync(c->d_buf.p, buf, buf_len, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_batches.p, batches, n * sizeof(grw_batch), hipMemcpyHostToDevice, c->stream));
  size_t nm = 0, ne = 0;
  if ((r = grow(c->d_msgs, msg_cap * sizeof(grw_message))) || (r = grow(c->d_ents, ent_cap * sizeof(grw_entry))))
    return r;
  r = grw_decode_device(c, (const u8*)c->d_buf.p, buf_len, (grw_batch*)c->d_batches.p, n, (grw_message*)c->d_msgs.p,
                        msg_cap, (grw_entry*)c->d_ents.p, ent_cap, &nm, &ne);
  *n_msgs = nm;
  *n_ents = ne;
  if (r) return r;
  HIPCHK(hipMemcpyAsync(batches, c->d_batches.p, n * sizeof(grw_batch), hipMemcpyDeviceToHost, c->stream));
  if (nm) HIPCHK(hipMemcpyAsync(msgs, c->d_msgs.p, nm * sizeof(grw_message), hipMemcpyDeviceToHost, c->stream));
  if (ne) HIPCHK(hipMemcpyAsync(ents, c->d_ents.p, ne * sizeof(grw_entry), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return GR_OK;
}

int grw_encode_device(grw_ctx* c, const uint8_t* d_payload, size_t payload_len, grw_batch* d_batches, size_t n,
                      const grw_message* d_msgs, size_t n_msgs, const grw_entry* d_ents, size_t n_ents, uint8_t* d_out,
                      size_t out_cap, size_t* out_len) {
  if (!c || !out_len || (n && !d_batches) || n > 0xFFFFFFFFull || n_msgs > 0xFFFFFFFFull) return GR_EINVAL;
  if ((n_msgs && !d_msgs) || (n_ents && !d_ents)) return GR_EINVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);  // shares scratch, stream and events with every other call
  *out_len = 0;
  if (n == 0) return GR_OK;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  int r;
  if ((r = grow(c->fsz, n_msgs * 8 + 8)) || (r = grow(c->pos, n_msgs * 8 + 16)) || (r = grow(c->flen, n * 8)) ||
      (r = grow(c->foff, n * 8 + 8)) || (r = grow(c->msg_batch, n_msgs * 4 + 4)) || (r = grow(c->pflag, n * 4)) ||
      (r = grow(c->scal, 64)))
    return r;
  EncScratch es{(u64*)c->fsz.p, (u64*)c->pos.p, (u64*)c->flen.p, (u64*)c->foff.p, (u32*)c->msg_batch.p,
                (u32*)c->scal.p};
  u32* pflag = (u32*)c->pflag.p;
  u32 total = (u32)n_msgs;
  HIPCHK(hipEventRecord(c->ev[0], s));
  HIPCHK(hipMemsetAsync(es.bad, 0, 4, s));
  check_contig<<<nblk(n, 256), 256, 0, s>>>(d_batches, (u32)n, total, es);
  check_records<<<nblk(std::max<u64>(std::max<u64>(n, total), n_ents), 256), 256, 0, s>>>(
      d_batches, (u32)n, d_msgs, total, d_ents, (u64)n_ents, (u64)payload_len, es);
  enc_map<<<(unsigned)n, 64, 0, s>>>(d_batches, (u32)n, total, es, pflag);
  HIPCHK(hipMemcpyAsync(c->h_scal, es.bad, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (((u32*)c->h_scal)[0]) return GR_EINVAL;
  HIPCHK(hipEventRecord(c->ev[1], s));
  if (total) {
    size_msgs<<<nblk(total, 256), 256, 0, s>>>(d_msgs, total, d_ents, es, pflag);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipMemsetAsync(es.fsz + total, 0, 8, s));
  if ((r = scan_excl<u64>(c, es.fsz, es.pos, (size_t)total + 1))) return r;
  frame_sizes<<<nblk(n, 256), 256, 0, s>>>(d_batches, (u32)n, es, pflag);
  if ((r = scan_excl<u64>(c, es.flen, es.foff, n))) return r;
  frame_finish<<<nblk(n, 256), 256, 0, s>>>(d_batches, (u32)n, es, pflag);
  HIPCHK(hipMemcpyAsync(c->h_scal, es.foff + n - 1, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(c->h_scal + 8, es.flen + n - 1, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(c->h_scal + 16, es.bad, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipEventRecord(c->ev[2], s));
  HIPCHK(hipStreamSynchronize(s));
  if (*(u32*)(c->h_scal + 16)) return GR_EINVAL;  // a frame longer than 2^32 - 1 bytes
  u64 need = ((u64*)c->h_scal)[0] + ((u64*)c->h_scal)[1];
  *out_len = need;
  if (need > out_cap || (need && !d_out)) return GR_ECAPACITY;
  HIPCHK(hipEventRecord(c->ev[3], s));
  if (total) write_msgs<<<nblk(total, 256), 256, 0, s>>>(d_batches, d_msgs, total, d_ents, d_payload, es, pflag, d_out);
  write_tails<<<nblk(n, 256), 256, 0, s>>>(d_batches, (u32)n, d_payload, es, pflag, d_out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ev[4], s));
  HIPCHK(hipStreamSynchronize(s));
  float t01 = 0, t12 = 0, t34 = 0, t04 = 0;
  hipEventElapsedTime(&t01, c->ev[0], c->ev[1]);
  hipEventElapsedTime(&t12, c->ev[1], c->ev[2]);
  hipEventElapsedTime(&t34, c->ev[3], c->ev[4]);
  hipEventElapsedTime(&t04, c->ev[0], c->ev[4]);
  c->timing = grw_timing{t01, 0.f, t12, t34, t04};
  return GR_OK;
}

int grw_encode(grw_ctx* c, const uint8_t* payload, size_t payload_len, grw_batch* batches, size_t n,
               const grw_message* msgs, size_t n_msgs, const grw_entry* ents, size_t n_ents, uint8_t* out,
               size_t out_cap, size_t* out_len) {
  if (!c || !out_len || (n && !batches)) return GR_EINVAL;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  int r;
  if ((r = grow(c->d_buf, payload_len + 16)) || (r = grow(c->d_batches, n * sizeof(grw_batch))) ||
      (r = grow(c->d_msgs, n_msgs * sizeof(grw_message))) || (r = grow(c->d_ents, n_ents * sizeof(grw_entry))))
    return r;
  if (payload_len) HIPCHK(hipMemcpyAsync(c->d_buf.p, payload, payload_len, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_batches.p, batches, n * sizeof(grw_batch), hipMemcpyHostToDevice, c->stream));
  if (n_msgs) HIPCHK(hipMemcpyAsync(c->d_msgs.p, msgs, n_msgs * sizeof(grw_message), hipMemcpyHostToDevice, c->stream));
  if (n_ents) HIPCHK(hipMemcpyAsync(c->d_ents.p, ents, n_ents * sizeof(grw_entry), hipMemcpyHostToDevice, c->stream));
  // size first (no output buffer), then the device output, then one DMA back
  size_t need = 0;
  r = grw_encode_device(c, (const u8*)c->d_buf.p, payload_len, (grw_batch*)c->d_batches.p, n,
                        (const grw_message*)c->d_msgs.p, n_msgs, (const grw_entry*)c->d_ents.p, n_ents, nullptr, 0,
                        &need);
  *out_len = need;
  if (r && r != GR_ECAPACITY) return r;
  if (need > out_cap) return GR_ECAPACITY;
  grw_ctx::Buf& dout = c->spans;  // reuse: decode scratch is idle during an encode
  if ((r = grow(dout, need + 16))) return r;
  r = grw_encode_device(c, (const u8*)c->d_buf.p, payload_len, (grw_batch*)c->d_batches.p, n,
                        (const grw_message*)c->d_msgs.p, n_msgs, (const grw_entry*)c->d_ents.p, n_ents, (u8*)dout.p,
                        need, &need);
  if (r) return r;
  HIPCHK(hipMemcpyAsync(batches, c->d_batches.p, n * sizeof(grw_batch), hipMemcpyDeviceToHost, c->stream));
  if (need) HIPCHK(hipMemcpyAsync(out, dout.p, need, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return GR_OK;
}

int grw_last_timing(grw_ctx* c, grw_timing* out) {
  if (!c || !out) return GR_EINVAL;
  *out = c->timing;
  return GR_OK;
}

}  // extern "C"
