"""numpy / ctypes mirrors of include/gpuraft.h (the C-ABI of libgpuraft.so).

The record layouts here must match the C structs byte for byte; the
``-m "not gpu"`` tests check every size against the library's expectations.
"""
import ctypes

import numpy as np

GR_K = 4
GR_Q = 4
GR_C = 6
GR_SMAX = 8
GR_SLOT_NONE = 0xFF

# raftpb/raft.pb.go:26-50
LOCAL_TICK, ELECTION, LEADER_HEARTBEAT, CONFIG_CHANGE_EVENT, NOOP, PING, PONG, PROPOSE = range(8)
SNAPSHOT_STATUS, UNREACHABLE, CHECK_QUORUM, BATCHED_READ_INDEX, REPLICATE, REPLICATE_RESP = range(8, 14)
REQUEST_VOTE, REQUEST_VOTE_RESP, INSTALL_SNAPSHOT, HEARTBEAT, HEARTBEAT_RESP = range(14, 19)
READ_INDEX, READ_INDEX_RESP, QUIESCE, SNAPSHOT_RECEIVED, LEADER_TRANSFER, TIMEOUT_NOW = range(19, 25)

MSG_NAMES = {
    0: "LocalTick", 1: "Election", 2: "LeaderHeartbeat", 3: "ConfigChangeEvent", 4: "NoOP",
    5: "Ping", 6: "Pong", 7: "Propose", 8: "SnapshotStatus", 9: "Unreachable", 10: "CheckQuorum",
    11: "BatchedReadIndex", 12: "Replicate", 13: "ReplicateResp", 14: "RequestVote",
    15: "RequestVoteResp", 16: "InstallSnapshot", 17: "Heartbeat", 18: "HeartbeatResp",
    19: "ReadIndex", 20: "ReadIndexResp", 21: "Quiesce", 22: "SnapshotReceived",
    23: "LeaderTransfer", 24: "TimeoutNow",
}

FOLLOWER, CANDIDATE, LEADER, OBSERVER = 0, 1, 2, 3
RETRY, WAIT, REPLICATE_ST, SNAPSHOT_ST = 0, 1, 2, 3
SLOT_EMPTY, SLOT_VOTER, SLOT_OBSERVER = 0, 1, 2
F_CHECK_QUORUM, F_IS_LEADER_TRANSFER_TARGET, F_PENDING_CONFIG_CHANGE = 1, 2, 4
PROP_NONE, PROP_APPENDED, PROP_DROPPED, PROP_FORWARDED = 0, 1, 2, 3

ESC_NAMES = ["none", "term_window", "random", "unsupported", "election", "panic", "capacity",
             "snapshot", "entry_size", "msg_runs", "nonmember", "config_change", "wide_term"]

u8, u32, u64 = np.uint8, np.uint32, np.uint64

REMOTE = np.dtype([("match", u64), ("next", u64), ("snapshot_index", u64), ("state", u8),
                   ("active", u8), ("kind", u8), ("pad", u8, (5,))])
READ_STATUS = np.dtype([("index", u64), ("ctx_low", u64), ("ctx_high", u64), ("from_slot", u8),
                        ("ack_bits", u8), ("pad", u8, (6,))])
PEER = np.dtype([
    ("term", u64), ("vote", u64), ("committed", u64), ("applied", u64), ("last_index", u64),
    ("first_index_m1", u64), ("leader_id", u64), ("leader_transfer_target", u64), ("node_id", u64),
    ("election_tick", u64), ("heartbeat_tick", u64), ("randomized_election_timeout", u64),
    ("election_timeout", u64), ("heartbeat_timeout", u64), ("entry_size_ub", u64),
    ("saved_to", u64), ("marker_index", u64), ("log_applied", u64),
    ("run_start", u64, (GR_K,)), ("run_term", u64, (GR_K,)), ("remote_id", u64, (GR_SMAX,)),
    ("remotes", REMOTE, (GR_SMAX,)), ("read_index", READ_STATUS, (GR_Q,)),
    ("state", u8), ("n_runs", u8), ("self_slot", u8), ("flags", u8), ("read_index_count", u8),
    ("pad", u8, (3,)),
])
MESSAGE = np.dtype([
    ("peer", u32), ("type", u8), ("slot", u8), ("reject", u8), ("n_runs", u8),
    ("n_entries", u32), ("run2_offset", u32),
    ("term", u64), ("log_index", u64), ("log_term", u64), ("commit", u64), ("hint", u64),
    ("hint_high", u64), ("run_term", u64, (2,)),
])
LOCAL = np.dtype([
    ("peer", u32), ("ticks", u32), ("quiesced_ticks", u32), ("propose_entries", u32),
    ("read_index", u8), ("propose_has_config_change", u8), ("pad", u8, (6,)),
    ("read_ctx_low", u64), ("read_ctx_high", u64), ("rand", u64),
])
READY = np.dtype([("index", u64), ("ctx_low", u64), ("ctx_high", u64)])
RESULT = np.dtype([
    ("peer", u32), ("escalation", u8), ("propose_result", u8), ("n_ready", u8), ("n_forwarded", u8),
    ("esc_item", u32), ("forwarded_entries", u32), ("append_from", u64), ("propose_first", u64),
    ("committed", u64), ("last_index", u64), ("save_from", u64), ("term", u64), ("vote", u64),
    ("ready", READY, (GR_Q,)),
])
# Compact boundary records (gr_step_compact)
CM_REJECT, CM_ENTRY, CM_LOG_TERM, CM_COMMIT, CM_HINT, CM_EXT = 0x01, 0x02, 0x04, 0x08, 0x10, 0x80
CM_ENTRY2, CM_PAIR = 0x20, 0x40  # a record standing for two messages (gpuraft.h GR_CM_PAIR)
CL_CONFIG_CHANGE, CL_EXT = 0x01, 0x80
CR_EXT = 0x80
CMSG = np.dtype([("peer", u32), ("type", u8), ("slot", u8), ("flags", u8), ("pad", u8), ("term", u32),
                 ("aux", u32), ("log_index", u64)])
CLOCAL = np.dtype([("peer", u32), ("propose_entries", u32), ("ticks", np.uint16), ("quiesced_ticks", u8),
                   ("flags", u8), ("ext", u32), ("rand", u64)])
CRESULT = np.dtype([("peer", u32), ("escalation", u8), ("propose_result", u8), ("flags", u8), ("save_count", u8),
                    ("aux", u32), ("commit_lag", u32), ("last_index", u64)])
assert CMSG.itemsize == 24 and CLOCAL.itemsize == 24 and CRESULT.itemsize == 24
UPDATE_COMMIT = np.dtype([("stable_log_to", u64), ("stable_log_term", u64), ("applied_to", u64)])
SIZES = {"gr_peer": 664, "gr_message": 80, "gr_local_input": 48, "gr_peer_result": 168,
         "gr_remote": 32, "gr_read_status": 32}
assert PEER.itemsize == SIZES["gr_peer"], PEER.itemsize
assert MESSAGE.itemsize == SIZES["gr_message"], MESSAGE.itemsize
assert LOCAL.itemsize == SIZES["gr_local_input"], LOCAL.itemsize
assert RESULT.itemsize == SIZES["gr_peer_result"], RESULT.itemsize


class Config(ctypes.Structure):
    _fields_ = [("max_peers", ctypes.c_uint32), ("slots", ctypes.c_uint32),
                ("window_runs", ctypes.c_uint32), ("read_index_depth", ctypes.c_uint32),
                ("mailbox_depth", ctypes.c_uint32), ("device", ctypes.c_uint32),
                ("max_entry_size", ctypes.c_uint64)]


class Inbox(ctypes.Structure):
    _fields_ = [("msgs", ctypes.c_void_p), ("n_msgs", ctypes.c_size_t),
                ("locals", ctypes.c_void_p), ("n_locals", ctypes.c_size_t)]


class Outbox(ctypes.Structure):
    _fields_ = [("msgs", ctypes.c_void_p), ("n_msgs", ctypes.c_size_t),
                ("results", ctypes.c_void_p), ("n_results", ctypes.c_size_t)]


class WireUnrouted(ctypes.Structure):
    _fields_ = [("n", ctypes.c_size_t), ("index", ctypes.c_void_p), ("reason", ctypes.c_void_p)]


WIRE_REASONS = ["routed", "no_peer", "nonmember", "snapshot", "type", "runs", "index"]


class CInbox(ctypes.Structure):
    _fields_ = [("msgs", ctypes.c_void_p), ("n_msgs", ctypes.c_size_t),
                ("ext_msgs", ctypes.c_void_p), ("n_ext_msgs", ctypes.c_size_t),
                ("locals", ctypes.c_void_p), ("n_locals", ctypes.c_size_t),
                ("ext_locals", ctypes.c_void_p), ("n_ext_locals", ctypes.c_size_t)]


class COutbox(ctypes.Structure):
    _fields_ = [("msgs", ctypes.c_void_p), ("n_msgs", ctypes.c_size_t),
                ("ext_msgs", ctypes.c_void_p), ("n_ext_msgs", ctypes.c_size_t),
                ("results", ctypes.c_void_p), ("n_results", ctypes.c_size_t),
                ("ext_results", ctypes.c_void_p), ("n_ext_results", ctypes.c_size_t)]


def cinbox_of(msgs, ext, locals_, lext):
    """A CInbox over numpy record arrays (kept alive by the caller)."""
    ib = CInbox()
    for name, a in (("msgs", msgs), ("ext_msgs", ext), ("locals", locals_), ("ext_locals", lext)):
        setattr(ib, name, a.ctypes.data if len(a) else None)
        setattr(ib, "n_" + name, len(a))
    return ib


class Stats(ctypes.Structure):
    _fields_ = [("passes", ctypes.c_uint64), ("leader_commits", ctypes.c_uint64),
                ("follower_commits", ctypes.c_uint64), ("escalations", ctypes.c_uint64),
                ("msgs_in", ctypes.c_uint64), ("msgs_out", ctypes.c_uint64),
                ("leader_msgs_in", ctypes.c_uint64), ("leader_msgs_out", ctypes.c_uint64),
                ("replicate_entries", ctypes.c_uint64)]


class Timing(ctypes.Structure):
    _fields_ = [("passes", ctypes.c_uint64), ("fast_ms", ctypes.c_double), ("general_ms", ctypes.c_double),
                ("bailed_lanes", ctypes.c_uint64)]


# settings.Soft.MaxEntrySize (internal/settings/soft.go:236)
MAX_ENTRY_SIZE = 2 * 32 * 1024 * 1024

# Every symbol include/gpuraft.h declares.
EXPORTS = [
    "gr_create", "gr_destroy", "gr_strerror", "gr_escalation_name", "gr_load_groups",
    "gr_sync_groups_to_host", "gr_step", "gr_inbox_reserve", "gr_release_outbox", "gr_stats_get", "gr_stats_reset",
    "gr_load_peers", "gr_sync_peers_to_host", "gr_notify_applied", "gr_compact_log", "gr_commit_update", "gr_space_bytes", "gr_space_chunk_bytes",
    "gr_space_hot_chunk_bytes", "gr_space_hot_tile_bytes", "gr_space_tile_positions", "gr_space_cold_used",
    "gr_space_side_bytes", "gr_space_side_pack", "gr_space_side_unpack", "gr_space_side_pack_host",
    "gr_space_side_unpack_host", "gr_space_cx_bytes", "gr_space_cx_pack", "gr_space_cx_unpack",
    "gr_space_cx_pack_host", "gr_space_cx_unpack_host", "gr_bind_routes",
    "gr_set_locals", "gr_step_device", "gr_step_compact", "gr_step_compact_begin", "gr_step_compact_end", "gr_cinbox_reserve", "gr_release_coutbox",
    "gr_pack_messages", "gr_unpack_messages", "gr_cmsg_count", "gr_pair_messages", "gr_pack_locals",
    "gr_collect_results", "gr_space_decode", "gr_space_encode", "gr_timing_begin", "gr_timing_end",
    "gr_bind_nodes", "gr_step_wire", "gr_step_wire_compact",
    "gr_graph_capture", "gr_graph_replay", "gr_graph_destroy",
]


def inbox_of(msgs, locals_):
    """Build an Inbox over numpy record arrays (kept alive by the caller)."""
    ib = Inbox()
    ib.msgs = msgs.ctypes.data if len(msgs) else None
    ib.n_msgs = len(msgs)
    ib.locals = locals_.ctypes.data if len(locals_) else None
    ib.n_locals = len(locals_)
    return ib
