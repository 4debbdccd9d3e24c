/*
 * gpuraft.h — C-ABI of libgpuraft.so, the MI355X batched Raft state-advance
 * engine (dragonboat_amd).
 *
 * Drop-in boundary for dragonboat's raft step path. In the reference, each
 * step worker (execengine.go:432-523) walks its ready clusters and calls
 * node.stepNode() (node.go:638-650), which drives raft.Peer one group at a
 * time: Peer.Handle per inbound message (peer.go:199-209), Peer.ReadIndex
 * (peer.go:262-269), Peer.Tick/QuiescedTick (peer.go:104-112) and
 * Peer.ProposeEntries (peer.go:126-134), in the order of node.handleEvents
 * (node.go:652-676) / handleReceivedMessages (node.go:746-780).
 * This library replaces that per-group loop (execengine.go:453-465) with one
 * device pass over every loaded group; a Go package internal/gpuraft binds it
 * through cgo. Plain C types only: no torch, no HIP types.
 *
 * Conventions:
 *  - int return: 0 = OK, negative = gr_error. Never aborts.
 *  - Inputs are caller-owned and read only during the call. Outbox arrays are
 *    engine-owned pinned memory, valid until gr_release_outbox() or the next
 *    gr_step() (the LookupDBStateMachine/FreeLookupResult pairing of
 *    internal/cpp/wrapper.go:242-258).
 *  - A reference invariant panic (e.g. logentry.go:284-287, readindex.go:55-58)
 *    never aborts here: the group escalates with GR_ESC_PANIC and the host
 *    re-runs that item with the unchanged Go code, which panics identically.
 *  - Peers are addressed by engine slot (0..max_peers-1). Remote nodes of a
 *    peer are addressed by remote slot (0..slots-1); the host keeps the
 *    slot <-> NodeID map (gr_peer.remote_id) and resolves m.From before
 *    packing, dropping responses from non-members as Peer.Handle does.
 */
#ifndef GPURAFT_H_
#define GPURAFT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Build-time capacities (a gr_config must match them). */
#define GR_K 4    /* term runs per group window (entryLog.term window) */
#define GR_Q 4    /* ReadIndex FIFO depth (readIndex.queue, readindex.go:31-34) */
#define GR_C 6    /* messages per (peer, remote slot) mailbox per pass (config 5 churn needs 5) */
#define GR_SMAX 8 /* remote slots per peer (voters + observers, incl. self) */
#define GR_SLOT_NONE 0xFF

/* raftpb/raft.pb.go:26-50 */
enum gr_msg_type {
  GR_LOCAL_TICK = 0, GR_ELECTION = 1, GR_LEADER_HEARTBEAT = 2, GR_CONFIG_CHANGE_EVENT = 3,
  GR_NOOP = 4, GR_PING = 5, GR_PONG = 6, GR_PROPOSE = 7, GR_SNAPSHOT_STATUS = 8,
  GR_UNREACHABLE = 9, GR_CHECK_QUORUM = 10, GR_BATCHED_READ_INDEX = 11, GR_REPLICATE = 12,
  GR_REPLICATE_RESP = 13, GR_REQUEST_VOTE = 14, GR_REQUEST_VOTE_RESP = 15,
  GR_INSTALL_SNAPSHOT = 16, GR_HEARTBEAT = 17, GR_HEARTBEAT_RESP = 18, GR_READ_INDEX = 19,
  GR_READ_INDEX_RESP = 20, GR_QUIESCE = 21, GR_SNAPSHOT_RECEIVED = 22,
  GR_LEADER_TRANSFER = 23, GR_TIMEOUT_NOW = 24
};

/* raft.go:58-66 */
enum gr_raft_state { GR_FOLLOWER = 0, GR_CANDIDATE = 1, GR_LEADER = 2, GR_OBSERVER = 3 };
/* remote.go:29-34 */
enum gr_remote_state { GR_RETRY = 0, GR_WAIT = 1, GR_REPLICATE_ST = 2, GR_SNAPSHOT_ST = 3 };
/* membership of a remote slot: raft.remotes (voter) / raft.observers */
enum gr_slot_kind { GR_SLOT_EMPTY = 0, GR_SLOT_VOTER = 1, GR_SLOT_OBSERVER = 2 };

/* gr_peer.flags */
#define GR_F_CHECK_QUORUM 0x01              /* raft.checkQuorum */
#define GR_F_IS_LEADER_TRANSFER_TARGET 0x02 /* raft.isLeaderTransferTarget */
#define GR_F_PENDING_CONFIG_CHANGE 0x04     /* raft.pendingConfigChange */

/* Why a group left the device fast path for the rest of a pass. */
enum gr_escalation {
  GR_ESC_NONE = 0,
  GR_ESC_TERM_WINDOW = 1,    /* term lookup below the device term window (LogReader.Term path) */
  GR_ESC_RANDOM = 2,         /* a second reset() in one pass needs another random draw */
  GR_ESC_UNSUPPORTED = 3,    /* message/state pair handled by the host (votes, snapshots, candidate) */
  GR_ESC_ELECTION = 4,       /* campaign() (raft.go:779-807) */
  GR_ESC_PANIC = 5,          /* the reference would panic on this item */
  GR_ESC_CAPACITY = 6,       /* mailbox / ReadIndex FIFO / ReadyToRead capacity */
  GR_ESC_SNAPSHOT = 7,       /* Replicate needs entries below firstIndex: InstallSnapshot path */
  GR_ESC_ENTRY_SIZE = 8,     /* settings.Soft.MaxEntrySize may bind (raft.go:513) */
  GR_ESC_MSG_RUNS = 9,       /* Replicate entries span more than 2 term runs */
  GR_ESC_NONMEMBER = 10,     /* target node id has no remote slot */
  GR_ESC_CONFIG_CHANGE = 11, /* proposal carries a ConfigChangeEntry (raft.go:1134-1143) */
  GR_ESC_WIDE_TERM = 12      /* a message term >= 2^32 (device mailboxes carry 32-bit terms) */
};

enum gr_error {
  GR_OK = 0,
  GR_EINVAL = -1,
  GR_ENOMEM = -2,
  GR_EDEVICE = -3,
  GR_ERANGE = -4,
  GR_ECAPACITY = -5,
  GR_ESTATE = -6
};

typedef struct gr_config {
  uint32_t max_peers;         /* engine slots */
  uint32_t slots;             /* remote slots per peer, 1..GR_SMAX (3 for R=3, 5 for R=5) */
  uint32_t window_runs;       /* must equal GR_K */
  uint32_t read_index_depth;  /* must equal GR_Q */
  uint32_t mailbox_depth;     /* must equal GR_C */
  uint32_t device;            /* HIP device ordinal */
  uint64_t max_entry_size;    /* settings.Soft.MaxEntrySize (soft.go:236) */
} gr_config;

/* remote.go:47-54 */
typedef struct gr_remote {
  uint64_t match, next, snapshot_index;
  uint8_t state;  /* gr_remote_state */
  uint8_t active; /* remote.active */
  uint8_t kind;   /* gr_slot_kind */
  uint8_t pad[5];
} gr_remote;

/* readindex.go:21-26; the confirmed map is a bitmap over remote slots */
typedef struct gr_read_status {
  uint64_t index, ctx_low, ctx_high;
  uint8_t from_slot; /* GR_SLOT_NONE = NoNode (local Peer.ReadIndex) */
  uint8_t ack_bits;  /* readStatus.confirmed */
  uint8_t pad[6];
} gr_read_status;

/*
 * Per-group state the device owns while the group is loaded: the fields of
 * raft (raft.go:124-154), entryLog (logentry.go:79-84) and the remotes that
 * the step path reads or writes. The log itself is represented by a term-run
 * window: runs (run_start[i], run_term[i]), i < n_runs, strictly increasing
 * starts, run i covering [run_start[i], run_start[i+1]) and the last run
 * covering up to last_index. term(index) is 0 outside [first_index_m1,
 * last_index] (logentry.go:141-145) and escalates below run_start[0].
 */
typedef struct gr_peer {
  uint64_t term, vote;
  uint64_t committed;      /* entryLog.committed */
  uint64_t applied;        /* raft.applied (NotifyRaftLastApplied), read by hasConfigChangeToApply */
  uint64_t last_index;     /* entryLog.lastIndex() */
  uint64_t first_index_m1; /* entryLog.firstIndex() - 1 */
  uint64_t leader_id, leader_transfer_target, node_id;
  uint64_t election_tick, heartbeat_tick, randomized_election_timeout;
  uint64_t election_timeout, heartbeat_timeout;
  uint64_t entry_size_ub;  /* upper bound of Entry.SizeUpperLimit() in this log (host-maintained) */
  /* The in-memory log's persistence marks (inmemory.go:29-34, logentry.go:78-83),
   * the state behind entriesToSave/commitUpdate:
   *   saved_to     inMemory.savedTo (entries <= saved_to are in LogDB)
   *   marker_index inMemory.markerIndex (first index kept in memory)
   *   log_applied  entryLog.applied (advanced by gr_commit_update)
   * marker_index == 0 means "a freshly loaded group" (newEntryLog,
   * logentry.go:86-95): the engine takes marker_index = last_index + 1,
   * saved_to = last_index, log_applied = first_index_m1. */
  uint64_t saved_to, marker_index, log_applied;
  uint64_t run_start[GR_K], run_term[GR_K];
  uint64_t remote_id[GR_SMAX];
  gr_remote remotes[GR_SMAX];
  gr_read_status read_index[GR_Q];
  uint8_t state;           /* gr_raft_state */
  uint8_t n_runs;
  uint8_t self_slot;       /* slot whose remote_id == node_id, GR_SLOT_NONE if self removed */
  uint8_t flags;           /* GR_F_* */
  uint8_t read_index_count;
  uint8_t pad[3];
} gr_peer;

/*
 * A step-path message (raftpb.Message, raft.pb.go:780-794, restricted to the
 * fields the step reads). Entries travel as term runs: entries have indexes
 * log_index+1 .. log_index+n_entries; entries [0, run2_offset) have term
 * run_term[0], entries [run2_offset, n_entries) have run_term[1]
 * (n_runs = 0 when n_entries = 0, 1 or 2 otherwise). Payloads stay host-side.
 */
typedef struct gr_message {
  uint32_t peer;       /* inbox: receiving engine slot; outbox: sending engine slot */
  uint8_t type;        /* gr_msg_type */
  uint8_t slot;        /* inbox: sender's remote slot; outbox: target remote slot */
  uint8_t reject;
  uint8_t n_runs;
  uint32_t n_entries;
  uint32_t run2_offset;
  uint64_t term, log_index, log_term, commit, hint, hint_high;
  uint64_t run_term[2];
} gr_message;

/* Per-pass local inputs of one peer, processed after its messages in the
 * order of node.handleReceivedMessages/handleEvents (node.go:652-780):
 * batched ReadIndex, ticks (clamped by the host to ElectionRTT, node.go:728),
 * quiesced ticks, then ProposeEntries. */
typedef struct gr_local_input {
  uint32_t peer;
  uint32_t ticks;          /* Peer.Tick() calls */
  uint32_t quiesced_ticks; /* Peer.QuiescedTick() calls after the normal ticks */
  uint32_t propose_entries;/* ProposeEntries batch size, 0 = none */
  uint8_t read_index;      /* Peer.ReadIndex(ctx) this pass */
  uint8_t propose_has_config_change;
  uint8_t pad[6];
  uint64_t read_ctx_low, read_ctx_high;
  uint64_t rand;           /* next random.LockGuardedRand.Uint64() draw for reset() */
} gr_local_input;

/* propose outcome */
enum gr_propose_result { GR_PROP_NONE = 0, GR_PROP_APPENDED = 1, GR_PROP_DROPPED = 2, GR_PROP_FORWARDED = 3 };

typedef struct gr_ready_to_read {
  uint64_t index, ctx_low, ctx_high;
} gr_ready_to_read;

typedef struct gr_peer_result {
  uint32_t peer;
  uint8_t escalation;      /* gr_escalation */
  uint8_t propose_result;  /* gr_propose_result */
  uint8_t n_ready;
  uint8_t n_forwarded;     /* Propose messages from remotes (handleFollowerPropose forwards) appended this pass */
  uint32_t esc_item;       /* first item NOT applied on device (messages, read index, ticks, qticks, propose) */
  uint32_t forwarded_entries; /* entries those n_forwarded batches appended */
  uint64_t append_from;    /* lowest index appended by Replicate this pass (0 = none): persist [append_from, last] */
  /* Index of the first entry a proposal appended this pass (0 = none). Proposals
   * append in item order and nothing else appends on a leader, so
   * [propose_first, propose_first + forwarded_entries) hold the forwarded
   * batches in arrival order (slot, then mailbox order) and the local
   * ProposeEntries batch, when propose_result == GR_PROP_APPENDED, follows. */
  uint64_t propose_first;
  /* The group's pb.Update fields after the items applied on the device
   * (getUpdate, peer.go:311-337): */
  uint64_t committed;      /* entryLog.committed: CommittedEntries end (start: log_applied + 1) */
  uint64_t last_index;     /* entryLog.lastIndex() */
  uint64_t save_from;      /* EntriesToSave = [save_from, last_index] (inMemory.entriesToSave,
                            * inmemory.go:101-108); 0 = nothing to save */
  uint64_t term, vote;     /* raftState(): pb.State{Term, Vote, Commit = committed} */
  gr_ready_to_read ready[GR_Q];
} gr_peer_result;

typedef struct gr_inbox {
  const gr_message* msgs;
  size_t n_msgs;
  const gr_local_input* locals;
  size_t n_locals;
} gr_inbox;

typedef struct gr_outbox {
  gr_message* msgs;        /* engine-owned */
  size_t n_msgs;
  gr_peer_result* results; /* one per peer that had input or produced output */
  size_t n_results;
} gr_outbox;

typedef struct gr_stats {
  uint64_t passes;
  uint64_t leader_commits;   /* leaders whose committed advanced, summed over passes */
  uint64_t follower_commits;
  uint64_t escalations;
  uint64_t msgs_in, msgs_out;
  uint64_t leader_msgs_in, leader_msgs_out; /* of lanes that ended the pass as leader */
  uint64_t replicate_entries;               /* sum of n over Replicate messages handled */
} gr_stats;

typedef struct gr_engine gr_engine;

/* Lifetime. */
int gr_create(const gr_config* cfg, gr_engine** out);
void gr_destroy(gr_engine* e);
const char* gr_strerror(int err);
const char* gr_escalation_name(int esc);

/* Load groups into engine slots [first, first+n) / read them back (the
 * loadBucketNodes hook, execengine.go:403-430, and the escalation hand-off). */
int gr_load_groups(gr_engine* e, uint32_t first, const gr_peer* peers, size_t n);
int gr_sync_groups_to_host(gr_engine* e, uint32_t first, gr_peer* out, size_t n);
/* The same for a list of engine slots (each listed once; GR_ERANGE for a slot
 * out of range or listed twice, before anything is written): the escalation
 * hand-off of scattered groups in one call, SURVEY.md §8b's
 * gr_sync_groups_to_host(cluster_ids) with ids already mapped to slots. */
int gr_load_peers(gr_engine* e, const uint32_t* slots, const gr_peer* peers, size_t n);
int gr_sync_peers_to_host(gr_engine* e, const uint32_t* slots, gr_peer* out, size_t n);

/* Peer.NotifyRaftLastApplied (peer.go:282-284) for a list of engine slots
 * (each listed once; GR_ERANGE before anything is written otherwise): sets
 * raft.applied, which handleNodeElection reads (raft.go:1055-1079). Call it
 * before each gr_step with the RSM's batched last applied index, as
 * node.handleEvents does first in every step (node.go:632-635,653). */
int gr_notify_applied(gr_engine* e, const uint32_t* slots, const uint64_t* applied, size_t n);

/* LogReader.Compact(index) (logreader.go:251-269) for a list of engine slots,
 * mirrored into entryLog.firstIndex()-1 (logentry.go:97-104): call it when the
 * host compacts a loaded group's LogDB range (node.compactLog). Per slot,
 * status (may be NULL) gets 0, 1 = ErrCompacted (index below firstIndex-1) or
 * 2 = ErrUnavailable (index past the persisted lastIndex, inMemory.savedTo:
 * LogReader's own range, not the unsaved in-memory tail); only status-0 slots are written
 * and the call returns GR_ESTATE if any slot was refused. Slots out of range or
 * listed twice: GR_ERANGE before anything is written. */
int gr_compact_log(gr_engine* e, const uint32_t* slots, const uint64_t* index, size_t n, int32_t* status);

/* entryLog.commitUpdate (logentry.go:325-335) for a list of engine slots: the
 * host reports what it persisted and applied after processing the pass's
 * pb.Update (node.processRaftUpdate -> Peer.Commit, peer.go:250-263):
 * inMemory.savedLogTo(stable_log_to, stable_log_term) when stable_log_to > 0,
 * then, when applied_to > 0, entryLog.applied = applied_to and
 * inMemory.appliedLogTo(applied_to) (inmemory.go:92-139). Snapshots stay on the
 * host (StableSnapshotTo: reload the group). Per slot, status (may be NULL):
 * 0 ok; 1 the reference panics ("invalid applyto": applied_to below
 * entryLog.applied or above committed); 2 the term of stable_log_to lies below
 * the device's term-run window (the host resolves it and reloads the group).
 * Refused slots are left untouched and the call returns GR_ESTATE. Slots out of
 * range or listed twice: GR_ERANGE before anything is written. */
typedef struct gr_update_commit {
  uint64_t stable_log_to, stable_log_term, applied_to;
} gr_update_commit;
int gr_commit_update(gr_engine* e, const uint32_t* slots, const gr_update_commit* uc, size_t n, int32_t* status);

/* One synchronous pass over host buffers (what a cgo caller uses). */
int gr_step(gr_engine* e, const gr_inbox* in, gr_outbox* out);
/* Engine-owned pinned buffers for the next gr_step's inbox: sets in->msgs /
 * in->locals to room for n_msgs / n_locals records and the counts to them. The
 * caller writes the records in place (no staging copy; the upload runs at
 * pinned-DMA rate) and passes `in` to gr_step. Valid until the next
 * gr_inbox_reserve or gr_destroy; gr_step may also be given any other memory. */
int gr_inbox_reserve(gr_engine* e, size_t n_msgs, size_t n_locals, gr_inbox* in);
int gr_release_outbox(gr_engine* e, gr_outbox* out);

/*
 * Compact records: the same pass as gr_step with the steady state's messages in
 * 24 bytes instead of 80, two of them per record where they repeat each other
 * (GR_CM_PAIR), and results in 24 bytes instead of 168, so a 1M-group pass moves
 * ~0.29 GB over PCIe instead of ~2 GB. A record that does not fit its compact
 * form points into an "ext" array of full records (GR_*_EXT); order is always
 * the compact array's. gr_pack_messages / gr_pair_messages / gr_unpack_messages
 * convert on the host (what a cgo caller's packer does).
 *
 * gr_cmsg: Term < 2^32; LogTerm, Commit, Hint and the entries follow from the
 * flags (fields not listed are 0): GR_CM_ENTRY = one entry at Term
 * (n_entries = n_runs = 1, run_term[0] = Term); GR_CM_LOG_TERM = LogTerm is Term;
 * GR_CM_COMMIT / GR_CM_HINT = Commit / Hint is LogIndex + aux - 2^31. Compact
 * Replicates, ReplicateResps, and Heartbeats / HeartbeatResps without a
 * ReadIndex context fit; everything else is GR_CM_EXT with ext index aux (the
 * ext record's peer, slot and type must equal the compact record's).
 */
#define GR_CM_REJECT 0x01
#define GR_CM_ENTRY 0x02
#define GR_CM_LOG_TERM 0x04
#define GR_CM_COMMIT 0x08
#define GR_CM_HINT 0x10
/* GR_CM_PAIR: the record stands for two consecutive messages of one mailbox
 * (same peer, slot, type and term), the steady state's usual pair: two
 * Replicates with the same LogIndex, LogTerm and Commit (a commit broadcast and
 * the proposal after it, makeReplicateMessage raft.go:474-498), the second
 * carrying one entry at Term when GR_CM_ENTRY2 is set; or two ReplicateResp
 * accepts, the second with LogIndex + 1 (their acks, raft.go:971-974). Replicate
 * transport batches a target's messages the same way (MessageBatch). */
#define GR_CM_ENTRY2 0x20
#define GR_CM_PAIR 0x40
#define GR_CM_EXT 0x80
typedef struct gr_cmsg {
  uint32_t peer;       /* as gr_message.peer */
  uint8_t type, slot, flags, pad;
  uint32_t term;
  uint32_t aux;        /* Commit/Hint offset from LogIndex (+2^31), or the ext index */
  uint64_t log_index;
} gr_cmsg;

/* gr_clocal: one peer's local inputs without a ReadIndex (GR_CL_EXT: ext_locals[ext]). */
#define GR_CL_CONFIG_CHANGE 0x01 /* gr_local_input.propose_has_config_change */
#define GR_CL_EXT 0x80
typedef struct gr_clocal {
  uint32_t peer;
  uint32_t propose_entries;
  uint16_t ticks;
  uint8_t quiesced_ticks;
  uint8_t flags;
  uint32_t ext;
  uint64_t rand;
} gr_clocal;

/* gr_cresult: a gr_peer_result without the per-pass extras, indexes relative
 * to last_index: committed = last_index - commit_lag; save_from = last_index -
 * save_count + 1, or 0 (nothing to save) when save_count is 0. GR_CR_EXT: the
 * lane has ReadyToRead records, forwarded proposals, a changed term/vote or an
 * escalation, or an index that does not fit (commit_lag >= 2^32, more than 255
 * entries to save), and ext_results[aux] is its full record; otherwise aux is
 * esc_item (0). propose_first (when propose_result is GR_PROP_APPENDED) is
 * last_index - propose_entries + 1. */
#define GR_CR_EXT 0x80
typedef struct gr_cresult {
  uint32_t peer;
  uint8_t escalation, propose_result, flags;
  uint8_t save_count;
  uint32_t aux;
  uint32_t commit_lag;
  uint64_t last_index;
} gr_cresult;

typedef struct gr_cinbox {
  const gr_cmsg* msgs;
  size_t n_msgs;
  const gr_message* ext_msgs;
  size_t n_ext_msgs;
  const gr_clocal* locals;
  size_t n_locals;
  const gr_local_input* ext_locals;
  size_t n_ext_locals;
} gr_cinbox;

typedef struct gr_coutbox { /* engine-owned pinned memory, as gr_outbox */
  gr_cmsg* msgs;
  size_t n_msgs;
  gr_message* ext_msgs;
  size_t n_ext_msgs;
  gr_cresult* results;
  size_t n_results;
  gr_peer_result* ext_results;
  size_t n_ext_results;
} gr_coutbox;

int gr_step_compact(gr_engine* e, const gr_cinbox* in, gr_coutbox* out);
/* gr_step_compact in two halves, so a step worker can overlap one partition's
 * upload with another's kernels and download (PCIe is full duplex): _begin
 * validates the inbox, copies it to the device and returns once the copy is
 * done (the inbox buffers may then be reused); _end runs the pass and fills
 * `out`. Every _begin is followed by exactly one _end on the same engine
 * (GR_EINVAL otherwise); another thread may call _end. Between the two the
 * pending pass owns the engine's scratch and lane rows: every other call on
 * that engine that steps it or uses them (gr_step, gr_step_compact{,_begin},
 * gr_step_device, gr_load_* / gr_sync_*, gr_set_locals, gr_bind_routes,
 * gr_compact_log, gr_commit_update, gr_notify_applied, gr_collect_results,
 * gr_space_cold_used) returns GR_ESTATE and changes nothing. */
int gr_step_compact_begin(gr_engine* e, const gr_cinbox* in);
int gr_step_compact_end(gr_engine* e, gr_coutbox* out);
/* Engine-owned pinned buffers for the next gr_step_compact inbox (as gr_inbox_reserve). */
int gr_cinbox_reserve(gr_engine* e, size_t n_msgs, size_t n_ext_msgs, size_t n_locals, size_t n_ext_locals,
                      gr_cinbox* in);
int gr_release_coutbox(gr_engine* e, gr_coutbox* out);
/* Host-side conversions (no engine): full records -> compact records plus ext
 * records (*n_ext of them, ext must have room for n), and back. */
int gr_pack_messages(const gr_message* in, size_t n, gr_cmsg* out, gr_message* ext, size_t* n_ext);
/* gr_unpack_messages writes gr_cmsg_count(in, n) records (a GR_CM_PAIR record
 * expands to two). gr_pair_messages merges, in place, each run of two
 * consecutive records that GR_CM_PAIR can carry (records that are not EXT);
 * *n_out = the records left. */
int gr_unpack_messages(const gr_cmsg* in, size_t n, const gr_message* ext, size_t n_ext, gr_message* out);
size_t gr_cmsg_count(const gr_cmsg* in, size_t n);
int gr_pair_messages(gr_cmsg* c, size_t n, size_t* n_out);
int gr_pack_locals(const gr_local_input* in, size_t n, gr_clocal* out, gr_local_input* ext, size_t* n_ext);
int gr_stats_get(gr_engine* e, gr_stats* out);
int gr_stats_reset(gr_engine* e);

/*
 * Per-kernel timing (benchmarks/profiling; not in the reference). Between
 * gr_timing_begin and gr_timing_end every pass records HIP events around its
 * kernels on the pass's stream: fast_ms brackets the lean kernels over all
 * lanes (steady kernel, role instances), general_ms the tail (tick and general
 * kernels) over the lanes the lean kernels handed over ("bailed").
 */
typedef struct gr_timing {
  uint64_t passes;
  double fast_ms;         /* summed over passes */
  double general_ms;
  uint64_t bailed_lanes;  /* summed over passes */
} gr_timing;
int gr_timing_begin(gr_engine* e);
int gr_timing_end(gr_engine* e, gr_timing* out);

/*
 * Device-resident path (benchmarks, multi-GPU exchange). Messages live in
 * "spaces": n_chunks chunks of `positions` mailboxes, each mailbox holding up
 * to `depth` (1..GR_C) messages in structure-of-arrays form; a lane that would
 * put more into one mailbox escalates GR_ESC_CAPACITY. Spaces that cross GPUs
 * use depth 2 (the steady state's two Replicates per follower per pass) and
 * move 2/GR_C of the bytes a full-depth space would. in_pos[j*max_peers+p] /
 * out_pos[j*max_peers+p] give the mailbox that peer p reads from / writes to
 * for remote slot j (0xFFFFFFFF = none). A chunk is one contiguous byte range,
 * so chunked spaces can be exchanged with one all-to-all.
 */
/* 0 when depth is not in 1..GR_C. A space is n_chunks hot chunks then n_chunks
 * cold chunks (gr_space_chunk_bytes = hot + cold per chunk): the hot region
 * holds the mailbox counts and every field of compact Replicates and non-reject
 * ReplicateResps, the cold region the rest. */
uint64_t gr_space_bytes(uint32_t n_chunks, uint32_t positions, uint32_t depth);
uint64_t gr_space_chunk_bytes(uint32_t positions, uint32_t depth);
uint64_t gr_space_hot_chunk_bytes(uint32_t positions, uint32_t depth);
/* A chunk's positions are tiled by W = gr_space_tile_positions(): tile t of its
 * hot region starts at t * gr_space_hot_tile_bytes(depth), and the tile's first
 * W bytes are the count bytes of positions Wt..Wt+W-1 (bit 3 set: the mailbox
 * needs no cold fields). 0 when depth is not in 1..GR_C. */
uint64_t gr_space_hot_tile_bytes(uint32_t depth);
/* Positions (and state slots) per tile: chunks hold a multiple of it. */
uint32_t gr_space_tile_positions(void);
/* *out = 1 when some mailbox of the (device) space holds a message with cold
 * fields, i.e. the cold region must travel with the hot one; runs on `stream`
 * and waits for it. */
int gr_space_cold_used(gr_engine* e, const void* space, uint32_t n_chunks, uint32_t positions, uint32_t depth,
                       void* stream, uint32_t* out);
/* Side buffers: how a space crosses GPUs without the host reading anything back
 * (dragonboat_amd/exchange.py Pipeline). The hot region travels every pass; the
 * cold fields travel only for the mailboxes that need them (count byte without
 * bit 3), compacted by gr_space_side_pack into `capacity` entries per chunk. A
 * mailbox that does not fit gets bit 4 (MB_COLD_LOST) in its count byte, and the
 * lane that reads it escalates GR_ESC_CAPACITY at its first message.
 * gr_space_side_unpack writes received entries into a space's cold chunks. Both
 * run on `stream` (a hipStream_t) without waiting for it; the _host forms run the
 * same codec over host memory (tests). gr_space_side_bytes: bytes of the side
 * buffers of n_chunks chunks (one range per chunk, in chunk order, 0 when depth
 * is not in 1..GR_C). The reference's role model: per-target message batching
 * (internal/transport/transport.go:399-476). */
uint64_t gr_space_side_bytes(uint32_t n_chunks, uint32_t depth, uint32_t capacity);
int gr_space_side_pack(void* space, uint32_t n_chunks, uint32_t positions, uint32_t depth, void* side,
                       uint32_t capacity, void* stream);
int gr_space_side_unpack(void* space, uint32_t n_chunks, uint32_t positions, uint32_t depth, const void* side,
                         uint32_t capacity, void* stream);
int gr_space_side_pack_host(void* space_host, uint32_t n_chunks, uint32_t positions, uint32_t depth,
                            void* side_host, uint32_t capacity);
int gr_space_side_unpack_host(void* space_host, uint32_t n_chunks, uint32_t positions, uint32_t depth,
                              const void* side_host, uint32_t capacity);
/* Compact exchange (round 5): the form in which a space crosses GPUs instead of
 * its whole hot region plus side buffers. Per chunk one fixed-size buffer
 * (gr_space_cx_bytes) carries only the mailboxes with messages: a 12-byte record
 * for a uniform mailbox whose messages repeat message 0's hot fields (one
 * message, or the steady state's shared pairs) and, round 6, for any mailbox of
 * up to three messages in a tick pass's or a commit advance's canonical forms
 * (a pattern record: Replicates at one LogIndex with Commits 0 or 1 apart,
 * accepts 0 or 1 apart, heartbeats and their acks with an empty context), a
 * full entry (hot fields and cold records) for any other, one bit for an empty
 * one. The buffer's header holds the packer's counters: records taken per
 * record region (16 regions, counters 64 B apart) and the full entries taken. capacities[c] records for
 * chunk c (at most 8 chunks) and `side_capacity` full entries per chunk; the
 * receiver passes the sender's capacities for its chunks. A mailbox that fits neither arrives as
 * lost (count 1 with bit 4, not uniform) and its reader escalates
 * GR_ESC_CAPACITY. gr_space_cx_pack reads a (device) out space into the buffers,
 * gr_space_cx_unpack writes received buffers into an in space (every count byte
 * of its chunks), both on `stream` without waiting; the _host forms run the same
 * codec over host memory (tests). The buffers of n_chunks chunks are one range
 * per chunk, in chunk order (an all-to-all's split sizes). The reference's model:
 * per-target batching of only the messages that exist
 * (internal/transport/transport.go:399-476). */
uint64_t gr_space_cx_bytes(uint32_t n_chunks, uint32_t positions, uint32_t depth, const uint32_t* capacities,
                           uint32_t side_capacity);
int gr_space_cx_pack(void* space, uint32_t n_chunks, uint32_t positions, uint32_t depth, void* cx,
                     const uint32_t* capacities, uint32_t side_capacity, void* stream);
int gr_space_cx_unpack(void* space, uint32_t n_chunks, uint32_t positions, uint32_t depth, const void* cx,
                       const uint32_t* capacities, uint32_t side_capacity, void* stream);
int gr_space_cx_pack_host(void* space_host, uint32_t n_chunks, uint32_t positions, uint32_t depth, void* cx_host,
                          const uint32_t* capacities, uint32_t side_capacity);
int gr_space_cx_unpack_host(void* space_host, uint32_t n_chunks, uint32_t positions, uint32_t depth,
                            const void* cx_host, const uint32_t* capacities, uint32_t side_capacity);
int gr_bind_routes(gr_engine* e, const uint32_t* in_pos, const uint32_t* out_pos, uint32_t n_peers);
int gr_set_locals(gr_engine* e, const gr_local_input* locals, size_t n);
/* Launch one pass on `stream` (a hipStream_t, may be NULL) without syncing.
 * in_space/out_space are device pointers laid out by gr_space_bytes() with
 * the same `depth`. */
int gr_step_device(gr_engine* e, const void* in_space, void* out_space, uint32_t in_chunks,
                   uint32_t in_positions, uint32_t out_chunks, uint32_t out_positions,
                   uint32_t depth, uint32_t n_peers, void* stream);
/* Graph mode (launch-bound small passes, e.g. BASELINE config 2):
 * gr_graph_capture records n_passes (even) device-resident passes over two
 * ping-pong spaces (pass k reads space_a when k is even, space_b when odd, and
 * writes the other) into a HIP graph with the engine's current routes and bound
 * local inputs; gr_graph_replay launches the whole sequence on `stream` with one
 * call, so a step worker that advances the same bound groups every tick
 * (execengine.go:453-465's per-group stepNode loop) pays one launch per
 * n_passes passes. Replays continue from the state the previous pass left (n_passes is
 * even, so every replay starts in space_a); gr_step_device calls may be mixed
 * in, in even numbers between replays (each pass flips the engine's counter and
 * hint sets and the live space): a replay at the other parity returns GR_ESTATE
 * and runs nothing. Capturing runs no pass and leaves the engine's pass count
 * and parities as they were. Capture refuses while per-pass timing is on
 * (GR_ESTATE); the spaces, routes and locals must stay as captured until
 * gr_graph_destroy. */
typedef struct gr_graph gr_graph;
int gr_graph_capture(gr_engine* e, void* space_a, void* space_b, uint32_t n_chunks, uint32_t positions,
                     uint32_t depth, uint32_t n_peers, uint32_t n_passes, gr_graph** out);
int gr_graph_replay(gr_graph* g, void* stream);
void gr_graph_destroy(gr_graph* g);
/* Copy per-peer results of the last device pass for peers [first, first+n). */
int gr_collect_results(gr_engine* e, uint32_t first, gr_peer_result* out, size_t n);
/* The wire path (SURVEY.md §8f-2 feeding the inbox): decoded raftpb.Message
 * records (gpuraft_wire.h grw_message / grw_entry, device pointers as
 * grw_decode_device leaves them in HBM) go straight into a gr_step pass, so the
 * frames are the only bytes that crossed PCIe on the way in. It replaces the
 * transport handing each message to its node (internal/transport/tcp.go:416-426
 * -> MessageBatch.Unmarshal raftpb/raft_optimized.go:1050 -> the node's queue)
 * and the host packing of gr_message records.
 * gr_bind_nodes: engine slot p is node node_ids[p] of cluster cluster_ids[p]
 * (n <= max_peers, every pair once). gr_step_wire routes every message by
 * (ClusterID, To) to its slot and by From to the sender's remote slot, turns its
 * entries into term runs, and runs gr_step's pass over the routed ones in wire
 * order (their arrival order) plus the host's local inputs. The messages it
 * cannot route stay with the host, listed in `unrouted` (engine-owned pinned
 * arrays valid until the next call): wire index and gr_wire_reason. */
enum gr_wire_reason {
  GR_WIRE_ROUTED = 0, GR_WIRE_NO_PEER = 1,    /* no slot holds (ClusterID, To) */
  GR_WIRE_NONMEMBER = 2,                       /* From is not a member (Peer.Handle, peer.go:200-209) */
  GR_WIRE_SNAPSHOT = 3,                        /* a non-zero Snapshot (InstallSnapshot: host) */
  GR_WIRE_TYPE = 4,                            /* not a type the engine steps */
  GR_WIRE_RUNS = 5,                            /* entries span more than two term runs */
  GR_WIRE_INDEX = 6                            /* a Replicate whose entries are not LogIndex+1.. */
};
typedef struct gr_wire_unrouted {
  size_t n;
  const uint32_t* index;  /* into the decoded message array */
  const uint8_t* reason;  /* gr_wire_reason */
} gr_wire_unrouted;
struct grw_message;
struct grw_entry;
int gr_bind_nodes(gr_engine* e, const uint64_t* cluster_ids, const uint64_t* node_ids, uint32_t n);
int gr_step_wire(gr_engine* e, const struct grw_message* d_msgs, size_t n_msgs, const struct grw_entry* d_ents,
                 size_t n_ents, const gr_local_input* locals, size_t n_locals, gr_outbox* out,
                 gr_wire_unrouted* unrouted);
/* gr_step_wire with the outbox and results as compact records (gr_coutbox, as
 * gr_step_compact returns them: 24-B gr_cmsg / 24-B gr_cresult, full records as
 * ext only where they do not fit); release with gr_release_coutbox. */
int gr_step_wire_compact(gr_engine* e, const struct grw_message* d_msgs, size_t n_msgs,
                         const struct grw_entry* d_ents, size_t n_ents, const gr_local_input* locals,
                         size_t n_locals, gr_coutbox* out, gr_wire_unrouted* unrouted);
/* Decode the messages of a device space into gr_message records (testing). A
 * mailbox whose cold fields were lost in the exchange (MB_COLD_LOST) decodes to
 * records with reject = 0xFF and no other field. */
int gr_space_decode(const void* space_host, uint32_t n_chunks, uint32_t positions, uint32_t depth,
                    gr_message* out, size_t cap, size_t* n_out);
int gr_space_encode(void* space_host, uint32_t n_chunks, uint32_t positions, uint32_t depth,
                    const gr_message* msgs, size_t n, const uint32_t* pos_of_msg);

#ifdef __cplusplus
}
#endif
#endif /* GPURAFT_H_ */
