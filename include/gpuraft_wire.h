/*
 * gpuraft_wire.h — C-ABI of libgrwire.so, the device codec for dragonboat's
 * raft wire format.
 *
 * Replaces, for a whole receive/send pass at once:
 *  - MessageBatch.Unmarshal      raftpb/raft_optimized.go:1050-1202 (called per
 *    frame at internal/transport/tcp.go:422), with Message.Unmarshal
 *    raft_optimized.go:653-977, Entry.unmarshal (colfer) :302-650,
 *    messageCount :1014-1048, entryCount :979-1012 and skipRaft
 *    raftpb/raft.pb.go:5139-5236;
 *  - MessageBatch.MarshalTo      raftpb/raft.pb.go:1929-1958 (called by
 *    sendMessageBatch, internal/transport/tcp.go), with Message.MarshalTo
 *    raft.pb.go:1747-1809, Entry.marshalTo raft_optimized.go:160-295 and the
 *    Size() functions raft.pb.go:2219-2320, raft_optimized.go:78-153.
 *
 * The decoded records describe the same values the Go structs would hold; byte
 * payloads (Entry.Cmd, MessageBatch.SourceAddress) are returned by reference
 * (offset + length into the input buffer), which is what a zero-copy Go binding
 * slices. A Message whose Snapshot field is not the zero Snapshot is flagged
 * (snapshot_host) and the host decodes that one message span with the Go code:
 * InstallSnapshot is rare and off the step path. The device does not validate
 * the Snapshot bytes, so for a frame holding a snapshot_host message the host's
 * re-decode of that span comes first: if the Go code rejects the Snapshot, that
 * error is the frame's error, whatever status the device reported for a later
 * message of the frame.
 *
 * A context runs one call at a time (host and device entry points alike share
 * its scratch, stream and events; calls from several threads serialise).
 *
 * Conventions as gpuraft.h: int return, 0 = OK, negative gr_error; never aborts.
 * A frame the reference would reject gets a per-batch status naming the Go
 * error (GRW_E_*); a frame on which the reference code itself panics (index out
 * of range inside messageCount/entryCount, or a slice bound overflow) gets
 * GRW_E_PANIC, and the Go shim panics as the reference does.
 */
#ifndef GPURAFT_WIRE_H_
#define GPURAFT_WIRE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GRW_COLFER_SIZE_MAX (256u * 1024u * 1024u) /* raft_optimized.go:31 */

/* Status of one MessageBatch.Unmarshal: the Go error it returns. */
enum grw_status {
  GRW_OK = 0,
  GRW_E_INT_OVERFLOW = 1,    /* ErrIntOverflowRaft, raft.pb.go:5241 */
  GRW_E_UNEXPECTED_EOF = 2,  /* io.ErrUnexpectedEOF */
  GRW_E_INVALID_LENGTH = 3,  /* ErrInvalidLengthRaft, raft.pb.go:5240 */
  GRW_E_END_GROUP = 4,       /* "proto: X: wiretype end group for non-group" */
  GRW_E_ILLEGAL_TAG = 5,     /* "proto: X: illegal tag %d" (field number <= 0) */
  GRW_E_WRONG_WIRE_TYPE = 6, /* "proto: wrong wireType = %d for field F" */
  GRW_E_ILLEGAL_WIRE_TYPE = 7, /* skipRaft: "proto: illegal wireType %d" */
  GRW_E_ENTRY_EOF = 8,       /* colfer io.EOF (Entry.unmarshal) */
  GRW_E_ENTRY_HEADER = 9,    /* ColferError: bad header byte */
  GRW_E_ENTRY_MAX = 10,      /* ColferMax: Cmd or entry above ColferSizeMax */
  GRW_E_PANIC = 11           /* the reference panics on this frame */
};

/* Where the error was raised. */
enum grw_err_level { GRW_LVL_BATCH = 0, GRW_LVL_MESSAGE = 1, GRW_LVL_ENTRY = 2 };

/* raftpb.MessageBatch (raft.pb.go:1133-1138); one per frame. */
typedef struct grw_batch {
  uint64_t deployment_id;
  uint64_t frame_off;   /* decode: input, frame offset in the buffer; encode: output, offset written */
  uint64_t source_off;  /* SourceAddress bytes: decode: offset in the input buffer; encode: in the payload buffer */
  uint32_t frame_len;   /* decode: input; encode: output, bytes written (MessageBatch.Size()) */
  uint32_t source_len;
  uint32_t first_msg;   /* decode: output; encode: input */
  uint32_t n_msgs;      /* decode: output (messages walked); encode: input */
  uint32_t bin_ver;
  int32_t status;       /* grw_status (decode output; encode: GRW_OK or GRW_E_PANIC) */
  uint32_t err_msg;     /* ordinal of the message (or of the next message, batch level) the error belongs to */
  uint32_t err_field;   /* field number of a wrong-wire-type / illegal-tag error, else 0 */
  uint8_t err_level;    /* grw_err_level */
  uint8_t pad[7];
} grw_batch;            /* 64 B */

/* raftpb.Message (raft.pb.go:780-794). */
typedef struct grw_message {
  uint64_t to, from, cluster_id, term, log_term, log_index, commit, hint, hint_high;
  uint64_t msg_off;       /* decode: offset of this Message's bytes in the input buffer */
  uint64_t snapshot_off;  /* decode: last Snapshot field's bytes; encode: marshalled Snapshot in the payload buffer */
  uint32_t msg_len;       /* decode: length of this Message's bytes */
  uint32_t snapshot_len;  /* encode: 0 = the zero Snapshot (its 12 canonical bytes are written) */
  uint32_t first_entry, n_entries;
  uint32_t batch;         /* decode: frame index */
  int32_t type;           /* raftpb.MessageType */
  uint8_t reject;
  uint8_t snapshot_host;  /* decode: Snapshot is not the zero value; decode [msg_off, +msg_len) on the host */
  uint8_t pad[6];
} grw_message;            /* 120 B */

/* raftpb.Entry (raft.pb.go:414-423); Cmd by reference. */
typedef struct grw_entry {
  uint64_t term, index, key, client_id, series_id, responded_to;
  uint64_t cmd_off;       /* decode: offset of Cmd in the input buffer; encode: in the payload buffer */
  uint32_t cmd_len;
  int32_t type;           /* raftpb.EntryType */
} grw_entry;              /* 64 B */

typedef struct grw_ctx grw_ctx;

typedef struct grw_timing {
  float walk_ms, scan_ms, message_ms, entry_ms, total_ms; /* device time of the last call's passes */
} grw_timing;

int grw_create(uint32_t device, grw_ctx** out);
void grw_destroy(grw_ctx* c);
const char* grw_status_name(int status);

/*
 * Decode n frames. batches[i].frame_off/frame_len name frame i inside buf (frames
 * must not overlap). On return every batch holds its fields and status; the
 * messages of frame i are msgs[first_msg .. first_msg+n_msgs) and the entries
 * of message j are ents[first_entry .. first_entry+n_entries), both in wire
 * order. Records of a failed frame are unspecified beyond its grw_batch. If the
 * totals exceed msg_cap / ent_cap, returns GR_ECAPACITY (-5) with *n_msgs /
 * *n_ents set to the totals needed and no records written.
 *
 * grw_decode takes host pointers (one DMA each way) and refuses (GR_EINVAL,
 * nothing decoded) a frame range outside buf or two frames that overlap;
 * grw_decode_device takes device pointers (inputs already in HBM), and only the
 * two totals cross PCIe: there the caller guarantees the frame ranges.
 */
int grw_decode(grw_ctx* c, const uint8_t* buf, size_t buf_len, grw_batch* batches, size_t n,
               grw_message* msgs, size_t msg_cap, grw_entry* ents, size_t ent_cap,
               size_t* n_msgs, size_t* n_ents);
int grw_decode_device(grw_ctx* c, const uint8_t* d_buf, size_t buf_len, grw_batch* d_batches, size_t n,
                      grw_message* d_msgs, size_t msg_cap, grw_entry* d_ents, size_t ent_cap,
                      size_t* n_msgs, size_t* n_ents);

/*
 * Encode n MessageBatch records: batch i holds msgs[first_msg .. +n_msgs); a
 * message's entries are ents[first_entry .. +n_entries); Cmd, SourceAddress and
 * non-zero Snapshot bytes come from payload. Frames are written back to back
 * into out; batches[i].frame_off/frame_len report where. Returns GR_ECAPACITY
 * with *out_len = the bytes needed when out_cap is too small. Every record is
 * checked on the device before any byte is read through it: a message's
 * entries past n_ents, or a Cmd / Snapshot / SourceAddress past payload_len,
 * and a frame longer than 2^32 - 1 bytes, return GR_EINVAL.
 */
int grw_encode(grw_ctx* c, const uint8_t* payload, size_t payload_len, grw_batch* batches, size_t n,
               const grw_message* msgs, size_t n_msgs, const grw_entry* ents, size_t n_ents,
               uint8_t* out, size_t out_cap, size_t* out_len);
int grw_encode_device(grw_ctx* c, const uint8_t* d_payload, size_t payload_len, grw_batch* d_batches,
                      size_t n, const grw_message* d_msgs, size_t n_msgs, const grw_entry* d_ents,
                      size_t n_ents, uint8_t* d_out, size_t out_cap, size_t* out_len);

int grw_last_timing(grw_ctx* c, grw_timing* out);

#ifdef __cplusplus
}
#endif
#endif /* GPURAFT_WIRE_H_ */
