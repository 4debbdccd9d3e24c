// wire_oracle.hpp — CPU restatement of dragonboat's raft wire codec.
//
// TEST INFRASTRUCTURE ONLY: the checker for libgrwire.so (include/gpuraft_wire.h).
// Only tests/, __graft_entry__.smoke() and tools/bench_wire.py's cpu_baseline leg
// load it; the product library never links it.
//
// Follows, reading the reference as text (Go is not in this image):
//   MessageBatch.Unmarshal   raftpb/raft_optimized.go:1050-1202
//   Message.Unmarshal        raftpb/raft_optimized.go:653-977
//   Entry.unmarshal (colfer) raftpb/raft_optimized.go:302-650
//   messageCount/entryCount  raftpb/raft_optimized.go:1014-1048 / 979-1012
//   skipRaft                 raftpb/raft.pb.go:5139-5236
//   MessageBatch.MarshalTo   raftpb/raft.pb.go:1929-1958, Size :2295-2311
//   Message.MarshalTo        raftpb/raft.pb.go:1747-1809, Size :2219-2245
//   Entry.marshalTo / Size   raftpb/raft_optimized.go:160-295 / 78-153
//   encodeVarintRaft / sov   raftpb/raft.pb.go:2058-2066 / 2347-2355
// Go integer semantics are kept: int is int64 with wrapping addition, shifts by
// >= the width give 0, and an index outside a slice is a panic (GRW_E_PANIC).
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

#include "gpuraft_wire.h"

namespace wire_oracle {

using u8 = uint8_t;
using u32 = uint32_t;
using i32 = int32_t;
using u64 = uint64_t;
using i64 = int64_t;

static inline i64 wrap_add(i64 a, i64 b) { return (i64)((u64)a + (u64)b); }

// The 12 bytes Snapshot{}.MarshalTo writes (raft.pb.go:1696-1735 with an empty
// Membership, raft.pb.go:1589-1594): Filepath "", FileSize 0, Index 0, Term 0,
// Membership{ConfigChangeId 0}.
static const u8 kZeroSnapshot[12] = {0x12, 0x00, 0x18, 0x00, 0x20, 0x00, 0x28, 0x00, 0x32, 0x02, 0x08, 0x00};

// ---------------------------------------------------------------- decode ----

// The bounds-checked varint of every generated field decoder
// (e.g. raft_optimized.go:658-671): shift >= 64 -> ErrIntOverflowRaft,
// index past the end -> io.ErrUnexpectedEOF.
static inline int rd_varint(const u8* d, i64 l, i64& i, u64& v) {
  v = 0;
  for (u32 shift = 0;; shift += 7) {
    if (shift >= 64) return GRW_E_INT_OVERFLOW;
    if (i >= l) return GRW_E_UNEXPECTED_EOF;
    u8 b = d[i++];
    v |= (u64)(b & 0x7F) << shift;
    if (b < 0x80) break;
  }
  return GRW_OK;
}

// The unchecked varint of messageCount/entryCount (raft_optimized.go:984-991):
// no shift limit, and d[i] outside the slice panics. Returns false on panic.
static inline bool rd_varint_nochk(const u8* d, i64 l, i64& i, u64& v) {
  v = 0;
  for (u64 shift = 0;; shift += 7) {
    if (i < 0 || i >= l) return false;
    u8 b = d[i++];
    if (shift < 64) v |= (u64)(b & 0x7F) << shift;
    if (b < 0x80) break;
  }
  return true;
}

// messageCount (field 1, raft_optimized.go:1014-1048) / entryCount (field 11,
// :979-1012) over d[0, l). Only a panic matters: the count sizes a capacity.
static inline bool count_chain_ok(const u8* d, i64 l, i32 field) {
  i64 i = 0;
  while (i < l) {
    u64 wire;
    if (!rd_varint_nochk(d, l, i, wire)) return false;
    if ((i32)(u32)(wire >> 3) != field) break;
    u64 len;
    if (!rd_varint_nochk(d, l, i, len)) return false;
    i = wrap_add(i, (i64)len);
  }
  return true;
}

// skipRaft (raft.pb.go:5139-5236) on d[0, l): returns the status and the bytes
// skipped. Start/end groups recurse in the reference; an explicit depth gives
// the same walk.
static inline int skip_raft(const u8* d, i64 l, i64& n) {
  i64 i = 0;
  u64 depth = 0;  // open groups
  for (;;) {
    // A length skipped inside a group can wrap i negative (Go int addition);
    // the next tag read then indexes dAtA[-k]: a panic.
    if (i < 0) return GRW_E_PANIC;
    u64 wire;
    int st = rd_varint(d, l, i, wire);
    if (st) return st;
    int wt = (int)(wire & 7);
    switch (wt) {
      case 0: {
        for (u32 shift = 0;; shift += 7) {
          if (shift >= 64) return GRW_E_INT_OVERFLOW;
          if (i >= l) return GRW_E_UNEXPECTED_EOF;
          i++;
          if (d[i - 1] < 0x80) break;
        }
        break;
      }
      case 1: i = wrap_add(i, 8); break;
      case 2: {
        u64 len;
        st = rd_varint(d, l, i, len);
        if (st) return st;
        i = wrap_add(i, (i64)len);
        if ((i64)len < 0) return GRW_E_INVALID_LENGTH;
        break;
      }
      case 3: depth++; break;
      case 4:
        // Only reached inside a group: the caller rejects a top-level end group.
        depth--;
        break;
      case 5: i = wrap_add(i, 4); break;
      default: return GRW_E_ILLEGAL_WIRE_TYPE;
    }
    if (depth == 0) {
      n = i;
      return GRW_OK;
    }
    // Inside a group the reference reads the next tag with bounds checks
    // (raft.pb.go:5190-5203); a field skipped past the end fails there.
  }
}

struct Err {
  int status = GRW_OK;
  int level = GRW_LVL_BATCH;
  u32 field = 0;
};

// Entry.unmarshal (raft_optimized.go:302-650) on d[0, l).
static inline int entry_unmarshal(const u8* d, i64 l, grw_entry& o, u64 base) {
  if (l == 0) return GRW_E_ENTRY_EOF;
  u8 header = d[0];
  i64 i = 1;
  u64* u64_field[7] = {&o.term, &o.index, nullptr, &o.key, &o.client_id, &o.series_id, &o.responded_to};
  for (int f = 0; f < 7; ++f) {
    if (f == 2) {  // Type, raft_optimized.go:379-436
      if (header == 2 || header == (2 | 0x80)) {
        if (i + 1 >= l) return GRW_E_ENTRY_EOF;
        u32 x = d[i];
        i++;
        if (x >= 0x80) {
          x &= 0x7f;
          for (u32 shift = 7;; shift += 7) {
            u32 b = d[i];
            i++;
            if (i >= l) return GRW_E_ENTRY_EOF;
            if (b < 0x80) {
              if (shift < 32) x |= b << shift;
              break;
            }
            if (shift < 32) x |= (b & 0x7f) << shift;
          }
        }
        o.type = (header == 2) ? (i32)x : (i32)(~x + 1);
        header = d[i];
        i++;
      }
      continue;
    }
    if (header == (u8)f) {  // varint form, e.g. raft_optimized.go:310-335
      i64 start = i;
      i++;
      if (i >= l) return GRW_E_ENTRY_EOF;
      u64 x = d[start];
      if (x >= 0x80) {
        x &= 0x7f;
        for (u32 shift = 7;; shift += 7) {
          u64 b = d[i];
          i++;
          if (i >= l) return GRW_E_ENTRY_EOF;
          if (b < 0x80 || shift == 56) {
            x |= b << shift;
            break;
          }
          x |= (b & 0x7f) << shift;
        }
      }
      *u64_field[f] = x;
      header = d[i];
      i++;
    } else if (header == (u8)(f | 0x80)) {  // fixed big-endian form, :336-345
      i64 start = i;
      i += 8;
      if (i >= l) return GRW_E_ENTRY_EOF;
      u64 x = 0;
      for (int k = 0; k < 8; ++k) x = (x << 8) | d[start + k];
      *u64_field[f] = x;
      header = d[i];
      i++;
    }
  }
  if (header == 7) {  // Cmd, raft_optimized.go:600-637
    if (i >= l) return GRW_E_ENTRY_EOF;
    u64 x = d[i];
    i++;
    if (x >= 0x80) {
      x &= 0x7f;
      for (u64 shift = 7;; shift += 7) {
        if (i >= l) return GRW_E_ENTRY_EOF;
        u64 b = d[i];
        i++;
        if (b < 0x80) {
          if (shift < 64) x |= b << shift;
          break;
        }
        if (shift < 64) x |= (b & 0x7f) << shift;
      }
    }
    if (x > (u64)GRW_COLFER_SIZE_MAX) return GRW_E_ENTRY_MAX;
    i64 start = i;
    i += (i64)x;
    if (i >= l) {
      if (i >= (i64)GRW_COLFER_SIZE_MAX) return GRW_E_ENTRY_MAX;  // eof label, :645-648
      return GRW_E_ENTRY_EOF;
    }
    o.cmd_off = base + (u64)start;
    o.cmd_len = (u32)x;
    header = d[i];
    i++;
  }
  if (header != 0x7f) return GRW_E_ENTRY_HEADER;
  if (i >= (i64)GRW_COLFER_SIZE_MAX) return GRW_E_ENTRY_MAX;
  return GRW_OK;
}

static inline bool is_zero_snapshot(const u8* d, i64 len) {
  return len == 0 || (len == 12 && memcmp(d, kZeroSnapshot, 12) == 0);
}

// Message.Unmarshal (raft_optimized.go:653-977) on d[0, l); d is buffer + base.
// Entries are appended to ents. A reference panic returns GRW_E_PANIC.
static inline Err message_unmarshal(const u8* d, i64 l, u64 base, grw_message& m, std::vector<grw_entry>& ents) {
  Err e;
  e.level = GRW_LVL_MESSAGE;
  i64 i = 0;
  bool have_entries = false;  // cap(m.Entries) != 0
  m.first_entry = (u32)ents.size();
  while (i < l) {
    i64 pre = i;
    u64 wire;
    if ((e.status = rd_varint(d, l, i, wire))) return e;
    i32 field = (i32)(u32)(wire >> 3);
    int wt = (int)(wire & 7);
    if (wt == 4) { e.status = GRW_E_END_GROUP; return e; }
    if (field <= 0) { e.status = GRW_E_ILLEGAL_TAG; e.field = (u32)field; return e; }
    if ((field >= 1 && field <= 10) || field == 13) {
      if (wt != 0) { e.status = GRW_E_WRONG_WIRE_TYPE; e.field = (u32)field; return e; }
      u64 v;
      if ((e.status = rd_varint(d, l, i, v))) return e;
      switch (field) {
        case 1: m.type = (i32)(u32)v; break;  // MessageType int32: low 32 bits
        case 2: m.to = v; break;
        case 3: m.from = v; break;
        case 4: m.cluster_id = v; break;
        case 5: m.term = v; break;
        case 6: m.log_term = v; break;
        case 7: m.log_index = v; break;
        case 8: m.commit = v; break;
        case 9: m.reject = v != 0; break;
        case 10: m.hint = v; break;
        case 13: m.hint_high = v; break;
      }
      continue;
    }
    if (field == 11 || field == 12) {
      if (wt != 2) { e.status = GRW_E_WRONG_WIRE_TYPE; e.field = (u32)field; return e; }
      u64 len;
      if ((e.status = rd_varint(d, l, i, len))) return e;
      if ((i64)len < 0) { e.status = GRW_E_INVALID_LENGTH; return e; }
      i64 post = wrap_add(i, (i64)len);
      if (post < 0) { e.status = GRW_E_PANIC; return e; }  // slice bounds out of range
      if (post > l) { e.status = GRW_E_UNEXPECTED_EOF; return e; }
      if (field == 11) {
        if (!have_entries) {  // m.entryCount(dAtA[postIndex:]), :883-886
          if (!count_chain_ok(d + post, l - post, 11)) { e.status = GRW_E_PANIC; return e; }
          have_entries = true;
        }
        grw_entry en;
        memset(&en, 0, sizeof(en));
        int st = entry_unmarshal(d + i, post - i, en, base + (u64)i);
        if (st) { e.status = st; e.level = GRW_LVL_ENTRY; return e; }
        ents.push_back(en);
      } else {
        if (!is_zero_snapshot(d + i, post - i)) m.snapshot_host = 1;
        m.snapshot_off = base + (u64)i;
        m.snapshot_len = (u32)(post - i);
      }
      i = post;
      continue;
    }
    // default: skipRaft, :955-968
    i = pre;
    i64 skippy;
    if ((e.status = skip_raft(d + i, l - i, skippy))) return e;
    if (skippy < 0) { e.status = GRW_E_INVALID_LENGTH; return e; }
    if (wrap_add(i, skippy) > l) { e.status = GRW_E_UNEXPECTED_EOF; return e; }
    i += skippy;
  }
  m.n_entries = (u32)ents.size() - m.first_entry;
  return e;
}

// MessageBatch.Unmarshal (raft_optimized.go:1050-1202) of one frame.
static inline void batch_unmarshal(const u8* buf, grw_batch& b, std::vector<grw_message>& msgs,
                                   std::vector<grw_entry>& ents, u32 batch_idx) {
  const u8* d = buf + b.frame_off;
  i64 l = b.frame_len;
  u64 base = b.frame_off;
  b.deployment_id = 0; b.source_off = 0; b.source_len = 0; b.bin_ver = 0;
  b.status = GRW_OK; b.err_msg = 0; b.err_field = 0; b.err_level = GRW_LVL_BATCH;
  b.first_msg = (u32)msgs.size();
  u32 n = 0;
  auto fail = [&](int st, int level, u32 field) {
    b.status = st; b.err_level = (u8)level; b.err_field = field; b.err_msg = n; b.n_msgs = n;
  };
  i64 i = 0;
  while (i < l) {
    i64 pre = i;
    u64 wire;
    int st = rd_varint(d, l, i, wire);
    if (st) return fail(st, GRW_LVL_BATCH, 0);
    i32 field = (i32)(u32)(wire >> 3);
    int wt = (int)(wire & 7);
    if (wt == 4) return fail(GRW_E_END_GROUP, GRW_LVL_BATCH, 0);
    if (field <= 0) return fail(GRW_E_ILLEGAL_TAG, GRW_LVL_BATCH, (u32)field);
    if (field == 1 || field == 3) {
      if (wt != 2) return fail(GRW_E_WRONG_WIRE_TYPE, GRW_LVL_BATCH, (u32)field);
      u64 len;
      if ((st = rd_varint(d, l, i, len))) return fail(st, GRW_LVL_BATCH, 0);
      if ((i64)len < 0) return fail(GRW_E_INVALID_LENGTH, GRW_LVL_BATCH, 0);
      i64 post = wrap_add(i, (i64)len);
      if (post < 0) return fail(GRW_E_PANIC, GRW_LVL_BATCH, 0);
      if (post > l) return fail(GRW_E_UNEXPECTED_EOF, GRW_LVL_BATCH, 0);
      if (field == 1) {
        if (n == 0 && !count_chain_ok(d + post, l - post, 1)) return fail(GRW_E_PANIC, GRW_LVL_BATCH, 0);
        grw_message m;
        memset(&m, 0, sizeof(m));
        m.batch = batch_idx;
        m.msg_off = base + (u64)i;
        m.msg_len = (u32)(post - i);
        Err e = message_unmarshal(d + i, post - i, base + (u64)i, m, ents);
        if (e.status) return fail(e.status, e.level, e.field);
        msgs.push_back(m);
        n++;
      } else {
        b.source_off = base + (u64)i;
        b.source_len = (u32)(post - i);
      }
      i = post;
      continue;
    }
    if (field == 2 || field == 4) {
      if (wt != 0) return fail(GRW_E_WRONG_WIRE_TYPE, GRW_LVL_BATCH, (u32)field);
      u64 v;
      if ((st = rd_varint(d, l, i, v))) return fail(st, GRW_LVL_BATCH, 0);
      if (field == 2) b.deployment_id = v; else b.bin_ver = (u32)v;
      continue;
    }
    i = pre;
    i64 skippy;
    if ((st = skip_raft(d + i, l - i, skippy))) return fail(st, GRW_LVL_BATCH, 0);
    if (skippy < 0) return fail(GRW_E_INVALID_LENGTH, GRW_LVL_BATCH, 0);
    if (wrap_add(i, skippy) > l) return fail(GRW_E_UNEXPECTED_EOF, GRW_LVL_BATCH, 0);
    i += skippy;
  }
  b.n_msgs = n;
}

// ---------------------------------------------------------------- encode ----

static inline int sov(u64 x) {  // sovRaft
  int n = 0;
  do { n++; x >>= 7; } while (x);
  return n;
}
static inline size_t put_varint(u8* d, size_t i, u64 v) {  // encodeVarintRaft
  while (v >= 0x80) { d[i++] = (u8)(v | 0x80); v >>= 7; }
  d[i++] = (u8)v;
  return i;
}

// Entry.Size (raft_optimized.go:78-153); returns -1 where it panics.
static inline i64 entry_size(const grw_entry& o) {
  i64 l = 1;
  const u64 f64[6] = {o.term, o.index, o.key, o.client_id, o.series_id, o.responded_to};
  for (int k = 0; k < 6; ++k) {
    u64 x = f64[k];
    if (x >= (1ull << 49)) l += 9;
    else if (x != 0) { for (l += 2; x >= 0x80; l++) x >>= 7; }
    if (k == 1 && o.type != 0) {
      u32 x32 = (u32)o.type;
      if (o.type < 0) x32 = ~x32 + 1;
      for (l += 2; x32 >= 0x80; l++) x32 >>= 7;
    }
  }
  if (u64 x = o.cmd_len) {
    if (x > GRW_COLFER_SIZE_MAX) return -1;
    for (l += (i64)x + 2; x >= 0x80; l++) x >>= 7;
  }
  if (l > (i64)GRW_COLFER_SIZE_MAX) return -1;
  return l;
}

// Entry.marshalTo (raft_optimized.go:160-295).
static inline size_t entry_marshal(u8* d, size_t i, const grw_entry& o, const u8* payload) {
  const u64 f64[6] = {o.term, o.index, o.key, o.client_id, o.series_id, o.responded_to};
  const u8 hdr[6] = {0, 1, 3, 4, 5, 6};
  for (int k = 0; k < 6; ++k) {
    u64 x = f64[k];
    if (x >= (1ull << 49)) {
      d[i] = hdr[k] | 0x80;
      for (int s = 0; s < 8; ++s) d[i + 1 + s] = (u8)(x >> (56 - 8 * s));
      i += 9;
    } else if (x != 0) {
      d[i++] = hdr[k];
      i = put_varint(d, i, x);
    }
    if (k == 1 && o.type != 0) {
      u32 x32 = (u32)o.type;
      if (o.type >= 0) d[i] = 2;
      else { x32 = ~x32 + 1; d[i] = 2 | 0x80; }
      i++;
      i = put_varint(d, i, x32);
    }
  }
  if (o.cmd_len != 0) {
    d[i++] = 7;
    i = put_varint(d, i, o.cmd_len);
    memcpy(d + i, payload + o.cmd_off, o.cmd_len);
    i += o.cmd_len;
  }
  d[i++] = 0x7f;
  return i;
}

static inline u64 snapshot_size(const grw_message& m) { return m.snapshot_len ? m.snapshot_len : 12; }

// Message.Size (raft.pb.go:2219-2245); -1 where an entry's Size panics.
static inline i64 message_size(const grw_message& m, const grw_entry* ents) {
  i64 n = 0;
  n += 1 + sov((u64)(i64)m.type);
  const u64 f[7] = {m.to, m.from, m.cluster_id, m.term, m.log_term, m.log_index, m.commit};
  for (u64 x : f) n += 1 + sov(x);
  n += 2;
  n += 1 + sov(m.hint);
  for (u32 k = 0; k < m.n_entries; ++k) {
    i64 l = entry_size(ents[m.first_entry + k]);
    if (l < 0) return -1;
    n += 1 + l + sov((u64)l);
  }
  u64 sl = snapshot_size(m);
  n += 1 + (i64)sl + sov(sl);
  n += 1 + sov(m.hint_high);
  return n;
}

// Message.MarshalTo (raft.pb.go:1747-1809).
static inline size_t message_marshal(u8* d, size_t i, const grw_message& m, const grw_entry* ents, const u8* payload) {
  d[i++] = 0x08; i = put_varint(d, i, (u64)(i64)m.type);
  d[i++] = 0x10; i = put_varint(d, i, m.to);
  d[i++] = 0x18; i = put_varint(d, i, m.from);
  d[i++] = 0x20; i = put_varint(d, i, m.cluster_id);
  d[i++] = 0x28; i = put_varint(d, i, m.term);
  d[i++] = 0x30; i = put_varint(d, i, m.log_term);
  d[i++] = 0x38; i = put_varint(d, i, m.log_index);
  d[i++] = 0x40; i = put_varint(d, i, m.commit);
  d[i++] = 0x48; d[i++] = m.reject ? 1 : 0;
  d[i++] = 0x50; i = put_varint(d, i, m.hint);
  for (u32 k = 0; k < m.n_entries; ++k) {
    const grw_entry& e = ents[m.first_entry + k];
    d[i++] = 0x5a;
    i = put_varint(d, i, (u64)entry_size(e));
    i = entry_marshal(d, i, e, payload);
  }
  d[i++] = 0x62;
  i = put_varint(d, i, snapshot_size(m));
  if (m.snapshot_len) { memcpy(d + i, payload + m.snapshot_off, m.snapshot_len); i += m.snapshot_len; }
  else { memcpy(d + i, kZeroSnapshot, 12); i += 12; }
  d[i++] = 0x68; i = put_varint(d, i, m.hint_high);
  return i;
}

// MessageBatch.Size (raft.pb.go:2295-2311); -1 where it panics.
static inline i64 batch_size(const grw_batch& b, const grw_message* msgs, const grw_entry* ents) {
  i64 n = 0;
  for (u32 k = 0; k < b.n_msgs; ++k) {
    i64 l = message_size(msgs[b.first_msg + k], ents);
    if (l < 0) return -1;
    n += 1 + l + sov((u64)l);
  }
  n += 1 + sov(b.deployment_id);
  n += 1 + (i64)b.source_len + sov(b.source_len);
  n += 1 + sov(b.bin_ver);
  return n;
}

// MessageBatch.MarshalTo (raft.pb.go:1929-1958).
static inline size_t batch_marshal(u8* d, size_t i, const grw_batch& b, const grw_message* msgs,
                                   const grw_entry* ents, const u8* payload) {
  for (u32 k = 0; k < b.n_msgs; ++k) {
    const grw_message& m = msgs[b.first_msg + k];
    d[i++] = 0x0a;
    i = put_varint(d, i, (u64)message_size(m, ents));
    i = message_marshal(d, i, m, ents, payload);
  }
  d[i++] = 0x10; i = put_varint(d, i, b.deployment_id);
  d[i++] = 0x1a; i = put_varint(d, i, b.source_len);
  memcpy(d + i, payload + b.source_off, b.source_len);
  i += b.source_len;
  d[i++] = 0x20; i = put_varint(d, i, b.bin_ver);
  return i;
}

}  // namespace wire_oracle
