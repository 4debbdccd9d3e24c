"""Python binding of libgpuraft.so (the product C-ABI, include/gpuraft.h).

This is the host-side mirror a Go ``internal/gpuraft`` package would be
(INTEGRATION.md): load groups, step them with messages and local inputs, read
back messages, results and state. The library is loaded from the in-tree
build (``dragonboat_amd/_build``); there is no fallback: if the HIP library
is missing or no GPU is usable, construction raises.
"""
import ctypes
import os

import numpy as np

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GPURAFT_LIB") or os.path.join(_HERE, "_build", "libgpuraft.so")  # env: A/B builds
_lib = None
_libs = {}  # other builds by path (e.g. the coverage build), loaded beside the default
MAILBOX_DEPTH = abi.GR_C  # full-depth spaces; exchange.py uses 2 for spaces that cross GPUs


class GpuRaftError(RuntimeError):
    pass


def load_library(path=LIB_PATH):
    """Load the HIP engine library (import torch first so one HIP runtime is shared)."""
    global _lib
    if path == LIB_PATH and _lib is not None:
        return _lib
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise GpuRaftError(f"libgpuraft.so not built at {path}; run __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    c = ctypes
    lib.gr_create.argtypes = [c.POINTER(abi.Config), c.POINTER(c.c_void_p)]
    lib.gr_destroy.argtypes = [c.c_void_p]
    lib.gr_destroy.restype = None
    lib.gr_strerror.restype = c.c_char_p
    lib.gr_strerror.argtypes = [c.c_int]
    lib.gr_escalation_name.restype = c.c_char_p
    lib.gr_escalation_name.argtypes = [c.c_int]
    lib.gr_load_groups.argtypes = [c.c_void_p, c.c_uint32, c.c_void_p, c.c_size_t]
    lib.gr_sync_groups_to_host.argtypes = [c.c_void_p, c.c_uint32, c.c_void_p, c.c_size_t]
    lib.gr_load_peers.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t]
    lib.gr_sync_peers_to_host.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t]
    lib.gr_notify_applied.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t]
    lib.gr_compact_log.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p]
    lib.gr_step_compact.argtypes = [c.c_void_p, c.POINTER(abi.CInbox), c.POINTER(abi.COutbox)]
    lib.gr_step_compact_begin.argtypes = [c.c_void_p, c.POINTER(abi.CInbox)]
    lib.gr_step_compact_end.argtypes = [c.c_void_p, c.POINTER(abi.COutbox)]
    lib.gr_cinbox_reserve.argtypes = [c.c_void_p, c.c_size_t, c.c_size_t, c.c_size_t, c.c_size_t,
                                      c.POINTER(abi.CInbox)]
    lib.gr_release_coutbox.argtypes = [c.c_void_p, c.POINTER(abi.COutbox)]
    lib.gr_pack_messages.argtypes = [c.c_void_p, c.c_size_t, c.c_void_p, c.c_void_p, c.POINTER(c.c_size_t)]
    lib.gr_unpack_messages.argtypes = [c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t, c.c_void_p]
    lib.gr_cmsg_count.argtypes = [c.c_void_p, c.c_size_t]
    lib.gr_cmsg_count.restype = c.c_size_t
    lib.gr_pair_messages.argtypes = [c.c_void_p, c.c_size_t, c.POINTER(c.c_size_t)]
    lib.gr_pack_locals.argtypes = [c.c_void_p, c.c_size_t, c.c_void_p, c.c_void_p, c.POINTER(c.c_size_t)]
    lib.gr_commit_update.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p]
    lib.gr_step.argtypes = [c.c_void_p, c.POINTER(abi.Inbox), c.POINTER(abi.Outbox)]
    lib.gr_release_outbox.argtypes = [c.c_void_p, c.POINTER(abi.Outbox)]
    lib.gr_inbox_reserve.argtypes = [c.c_void_p, c.c_size_t, c.c_size_t, c.POINTER(abi.Inbox)]
    lib.gr_stats_get.argtypes = [c.c_void_p, c.POINTER(abi.Stats)]
    lib.gr_stats_reset.argtypes = [c.c_void_p]
    lib.gr_space_bytes.restype = c.c_uint64
    lib.gr_space_bytes.argtypes = [c.c_uint32, c.c_uint32, c.c_uint32]
    lib.gr_space_chunk_bytes.restype = c.c_uint64
    lib.gr_space_chunk_bytes.argtypes = [c.c_uint32, c.c_uint32]
    lib.gr_space_hot_chunk_bytes.restype = c.c_uint64
    lib.gr_space_hot_chunk_bytes.argtypes = [c.c_uint32, c.c_uint32]
    lib.gr_space_hot_tile_bytes.restype = c.c_uint64
    lib.gr_space_hot_tile_bytes.argtypes = [c.c_uint32]
    lib.gr_space_tile_positions.restype = c.c_uint32
    lib.gr_space_tile_positions.argtypes = []
    lib.gr_space_cold_used.argtypes = [c.c_void_p, c.c_void_p, c.c_uint32, c.c_uint32, c.c_uint32, c.c_void_p,
                                       c.POINTER(c.c_uint32)]
    lib.gr_space_side_bytes.restype = c.c_uint64
    lib.gr_space_side_bytes.argtypes = [c.c_uint32, c.c_uint32, c.c_uint32]
    for f in ("gr_space_side_pack", "gr_space_side_unpack"):
        getattr(lib, f).argtypes = [c.c_void_p, c.c_uint32, c.c_uint32, c.c_uint32, c.c_void_p, c.c_uint32,
                                    c.c_void_p]
    for f in ("gr_space_side_pack_host", "gr_space_side_unpack_host"):
        getattr(lib, f).argtypes = [c.c_void_p, c.c_uint32, c.c_uint32, c.c_uint32, c.c_void_p, c.c_uint32]
    lib.gr_space_cx_bytes.restype = c.c_uint64
    lib.gr_space_cx_bytes.argtypes = [c.c_uint32, c.c_uint32, c.c_uint32, c.c_void_p, c.c_uint32]
    for f in ("gr_space_cx_pack", "gr_space_cx_unpack"):
        getattr(lib, f).argtypes = [c.c_void_p, c.c_uint32, c.c_uint32, c.c_uint32, c.c_void_p, c.c_void_p,
                                    c.c_uint32, c.c_void_p]
    for f in ("gr_space_cx_pack_host", "gr_space_cx_unpack_host"):
        getattr(lib, f).argtypes = [c.c_void_p, c.c_uint32, c.c_uint32, c.c_uint32, c.c_void_p, c.c_void_p,
                                    c.c_uint32]
    lib.gr_bind_routes.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_uint32]
    lib.gr_bind_nodes.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_uint32]
    lib.gr_step_wire.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t, c.c_void_p,
                                 c.c_size_t, c.POINTER(abi.Outbox), c.POINTER(abi.WireUnrouted)]
    lib.gr_step_wire_compact.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t, c.c_void_p,
                                         c.c_size_t, c.POINTER(abi.COutbox), c.POINTER(abi.WireUnrouted)]
    lib.gr_set_locals.argtypes = [c.c_void_p, c.c_void_p, c.c_size_t]
    lib.gr_step_device.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_uint32, c.c_uint32,
                                   c.c_uint32, c.c_uint32, c.c_uint32, c.c_uint32, c.c_void_p]
    lib.gr_collect_results.argtypes = [c.c_void_p, c.c_uint32, c.c_void_p, c.c_size_t]
    if hasattr(lib, "gr_graph_capture"):  # (older builds loaded for A/B runs lack graph mode)
        lib.gr_graph_capture.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_uint32, c.c_uint32, c.c_uint32,
                                         c.c_uint32, c.c_uint32, c.POINTER(c.c_void_p)]
        lib.gr_graph_replay.argtypes = [c.c_void_p, c.c_void_p]
        lib.gr_graph_destroy.argtypes = [c.c_void_p]
        lib.gr_graph_destroy.restype = None
    lib.gr_space_decode.argtypes = [c.c_void_p, c.c_uint32, c.c_uint32, c.c_uint32, c.c_void_p, c.c_size_t,
                                    c.POINTER(c.c_size_t)]
    lib.gr_space_encode.argtypes = [c.c_void_p, c.c_uint32, c.c_uint32, c.c_uint32, c.c_void_p, c.c_size_t,
                                    c.c_void_p]
    lib.gr_timing_begin.argtypes = [c.c_void_p]
    lib.gr_timing_end.argtypes = [c.c_void_p, c.POINTER(abi.Timing)]
    if hasattr(lib, "gr_coverage_read"):  # coverage build only (GR_COVERAGE)
        lib.gr_coverage_read.argtypes = [c.c_void_p, c.c_uint32]
        lib.gr_coverage_names.restype = c.c_char_p
    if path == LIB_PATH:
        _lib = lib
    _libs[path] = lib
    return lib


def _check(rc, what):
    if rc != 0:
        raise GpuRaftError(f"{what}: {load_library().gr_strerror(rc).decode()} ({rc})")


class Engine:
    """One engine = one device's slab of group slots (engine slots 0..max_peers-1)."""

    def __init__(self, max_peers, slots=3, device=0, max_entry_size=abi.MAX_ENTRY_SIZE, lib_path=None):
        lib = load_library(lib_path or LIB_PATH)
        cfg = abi.Config(max_peers=max_peers, slots=slots, window_runs=abi.GR_K,
                         read_index_depth=abi.GR_Q, mailbox_depth=abi.GR_C, device=device,
                         max_entry_size=max_entry_size)
        h = ctypes.c_void_p()
        _check(lib.gr_create(ctypes.byref(cfg), ctypes.byref(h)), "gr_create")
        self._h = h
        self.max_peers = max_peers
        self.slots = slots
        self.lib = lib

    def close(self):
        if self._h:
            self.lib.gr_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, peers, first=0):
        peers = np.ascontiguousarray(peers, dtype=abi.PEER)
        _check(self.lib.gr_load_groups(self._h, first, peers.ctypes.data, len(peers)), "gr_load_groups")

    def sync(self, n=None, first=0):
        n = self.max_peers - first if n is None else n
        out = np.zeros(n, dtype=abi.PEER)
        _check(self.lib.gr_sync_groups_to_host(self._h, first, out.ctypes.data, n), "gr_sync")
        return out

    def load_peers(self, slots, peers):
        """Load records into a list of engine slots (gr_load_peers)."""
        slots = np.ascontiguousarray(slots, np.uint32)
        peers = np.ascontiguousarray(peers, dtype=abi.PEER)
        assert len(slots) == len(peers)
        _check(self.lib.gr_load_peers(self._h, slots.ctypes.data if len(slots) else None,
                                      peers.ctypes.data if len(peers) else None, len(peers)), "gr_load_peers")

    def sync_peers(self, slots):
        """Records of a list of engine slots (gr_sync_peers_to_host)."""
        slots = np.ascontiguousarray(slots, np.uint32)
        out = np.zeros(len(slots), dtype=abi.PEER)
        _check(self.lib.gr_sync_peers_to_host(self._h, slots.ctypes.data if len(slots) else None,
                                              out.ctypes.data if len(out) else None, len(slots)),
               "gr_sync_peers_to_host")
        return out

    def notify_applied(self, slots, applied):
        """Peer.NotifyRaftLastApplied for a list of engine slots (gr_notify_applied)."""
        slots = np.ascontiguousarray(slots, np.uint32)
        applied = np.ascontiguousarray(applied, np.uint64)
        assert len(slots) == len(applied)
        _check(self.lib.gr_notify_applied(self._h, slots.ctypes.data if len(slots) else None,
                                          applied.ctypes.data if len(applied) else None, len(slots)),
               "gr_notify_applied")

    def compact_log(self, slots, index):
        """LogReader.Compact mirrored on the device (gr_compact_log); returns
        (rc, per-slot status: 0 ok, 1 ErrCompacted, 2 ErrUnavailable)."""
        slots = np.ascontiguousarray(slots, np.uint32)
        index = np.ascontiguousarray(index, np.uint64)
        assert len(slots) == len(index)
        st = np.zeros(len(slots), np.int32)
        rc = self.lib.gr_compact_log(self._h, slots.ctypes.data if len(slots) else None,
                                     index.ctypes.data if len(index) else None, len(slots),
                                     st.ctypes.data if len(st) else None)
        if rc not in (0, -6):
            _check(rc, "gr_compact_log")
        return rc, st

    def commit_update(self, slots, uc):
        """entryLog.commitUpdate on the device (gr_commit_update): uc is an
        abi.UPDATE_COMMIT array. Returns (rc, per-slot status: 0 ok, 1 the
        reference panics, 2 term below the device window)."""
        slots = np.ascontiguousarray(slots, np.uint32)
        uc = np.ascontiguousarray(uc, abi.UPDATE_COMMIT)
        assert len(slots) == len(uc)
        st = np.zeros(len(slots), np.int32)
        rc = self.lib.gr_commit_update(self._h, slots.ctypes.data if len(slots) else None,
                                       uc.ctypes.data if len(uc) else None, len(slots),
                                       st.ctypes.data if len(st) else None)
        if rc not in (0, -6):
            _check(rc, "gr_commit_update")
        return rc, st

    def step(self, msgs=None, locals_=None):
        """One synchronous pass (gr_step). Returns (messages, results) record arrays."""
        msgs = np.zeros(0, abi.MESSAGE) if msgs is None else np.ascontiguousarray(msgs, abi.MESSAGE)
        locals_ = np.zeros(0, abi.LOCAL) if locals_ is None else np.ascontiguousarray(locals_, abi.LOCAL)
        ib = abi.inbox_of(msgs, locals_)
        ob = abi.Outbox()
        _check(self.lib.gr_step(self._h, ctypes.byref(ib), ctypes.byref(ob)), "gr_step")
        out = np.zeros(ob.n_msgs, abi.MESSAGE)
        res = np.zeros(ob.n_results, abi.RESULT)
        if ob.n_msgs:
            ctypes.memmove(out.ctypes.data, ob.msgs, ob.n_msgs * abi.MESSAGE.itemsize)
        if ob.n_results:
            ctypes.memmove(res.ctypes.data, ob.results, ob.n_results * abi.RESULT.itemsize)
        _check(self.lib.gr_release_outbox(self._h, ctypes.byref(ob)), "gr_release_outbox")
        return out, res

    def bind_nodes(self, cluster_ids, node_ids):
        """gr_bind_nodes: engine slot p is node node_ids[p] of cluster cluster_ids[p]."""
        cl = np.ascontiguousarray(cluster_ids, np.uint64)
        nd = np.ascontiguousarray(node_ids, np.uint64)
        assert len(cl) == len(nd)
        _check(self.lib.gr_bind_nodes(self._h, cl.ctypes.data if len(cl) else None,
                                      nd.ctypes.data if len(nd) else None, len(cl)), "gr_bind_nodes")

    def step_wire(self, d_msgs, n_msgs, d_ents, n_ents, locals_=None, compact=False):
        """gr_step_wire over decoded wire records already in HBM (device pointers, as
        grw_decode_device leaves them). Returns (messages, results, unrouted
        indices, unrouted reasons); with compact=True gr_step_wire_compact, whose
        outbox is returned as step_compact returns it: ((cmsgs, ext msgs, cresults,
        ext results), unrouted indices, unrouted reasons)."""
        locals_ = np.zeros(0, abi.LOCAL) if locals_ is None else np.ascontiguousarray(locals_, abi.LOCAL)
        ob = abi.COutbox() if compact else abi.Outbox()
        un = abi.WireUnrouted()
        fn = self.lib.gr_step_wire_compact if compact else self.lib.gr_step_wire
        _check(fn(self._h, d_msgs, n_msgs, d_ents, n_ents, locals_.ctypes.data if len(locals_) else None,
                  len(locals_), ctypes.byref(ob), ctypes.byref(un)), fn.__name__)
        idx = np.zeros(un.n, np.uint32)
        why = np.zeros(un.n, np.uint8)
        if un.n:
            ctypes.memmove(idx.ctypes.data, un.index, un.n * 4)
            ctypes.memmove(why.ctypes.data, un.reason, un.n)
        if compact:
            return self._take_coutbox(ob), idx, why
        out = np.zeros(ob.n_msgs, abi.MESSAGE)
        res = np.zeros(ob.n_results, abi.RESULT)
        if ob.n_msgs:
            ctypes.memmove(out.ctypes.data, ob.msgs, ob.n_msgs * abi.MESSAGE.itemsize)
        if ob.n_results:
            ctypes.memmove(res.ctypes.data, ob.results, ob.n_results * abi.RESULT.itemsize)
        _check(self.lib.gr_release_outbox(self._h, ctypes.byref(ob)), "gr_release_outbox")
        return out, res, idx, why

    def pack_messages(self, msgs):
        """gr_pack_messages: full records -> (compact records, ext records)."""
        msgs = np.ascontiguousarray(msgs, abi.MESSAGE)
        c = np.zeros(len(msgs), abi.CMSG)
        ext = np.zeros(len(msgs), abi.MESSAGE)
        nx = ctypes.c_size_t()
        _check(self.lib.gr_pack_messages(msgs.ctypes.data if len(msgs) else None, len(msgs),
                                         c.ctypes.data if len(c) else None, ext.ctypes.data if len(ext) else None,
                                         ctypes.byref(nx)), "gr_pack_messages")
        return c, ext[:nx.value].copy()

    def pair_messages(self, c):
        """gr_pair_messages: compact records with every pair GR_CM_PAIR carries merged."""
        c = np.array(c, abi.CMSG)
        n = ctypes.c_size_t()
        _check(self.lib.gr_pair_messages(c.ctypes.data if len(c) else None, len(c), ctypes.byref(n)),
               "gr_pair_messages")
        return c[:n.value].copy()

    def unpack_messages(self, c, ext):
        """gr_unpack_messages: compact (and ext) records -> full records (a pair record -> two)."""
        c = np.ascontiguousarray(c, abi.CMSG)
        ext = np.ascontiguousarray(ext, abi.MESSAGE)
        out = np.zeros(int(self.lib.gr_cmsg_count(c.ctypes.data if len(c) else None, len(c))), abi.MESSAGE)
        _check(self.lib.gr_unpack_messages(c.ctypes.data if len(c) else None, len(c),
                                           ext.ctypes.data if len(ext) else None, len(ext),
                                           out.ctypes.data if len(out) else None), "gr_unpack_messages")
        return out

    def pack_locals(self, loc):
        loc = np.ascontiguousarray(loc, abi.LOCAL)
        c = np.zeros(len(loc), abi.CLOCAL)
        ext = np.zeros(len(loc), abi.LOCAL)
        nx = ctypes.c_size_t()
        _check(self.lib.gr_pack_locals(loc.ctypes.data if len(loc) else None, len(loc),
                                       c.ctypes.data if len(c) else None, ext.ctypes.data if len(ext) else None,
                                       ctypes.byref(nx)), "gr_pack_locals")
        return c, ext[:nx.value].copy()

    def step_compact(self, cmsgs, ext_msgs, clocals, ext_locals, halves=False):
        """One synchronous pass with compact records (gr_step_compact, or with
        halves=True its two halves gr_step_compact_begin + _end). Returns
        (cmsgs, ext msgs, cresults, ext results) copied out of the engine's outbox."""
        ib = abi.cinbox_of(cmsgs, ext_msgs, clocals, ext_locals)
        ob = abi.COutbox()
        if halves:
            _check(self.lib.gr_step_compact_begin(self._h, ctypes.byref(ib)), "gr_step_compact_begin")
            _check(self.lib.gr_step_compact_end(self._h, ctypes.byref(ob)), "gr_step_compact_end")
        else:
            _check(self.lib.gr_step_compact(self._h, ctypes.byref(ib), ctypes.byref(ob)), "gr_step_compact")
        return self._take_coutbox(ob)

    def _take_coutbox(self, ob):
        """(cmsgs, ext msgs, cresults, ext results) copied out of a gr_coutbox, released."""
        out = []
        for ptr, n, dt in ((ob.msgs, ob.n_msgs, abi.CMSG), (ob.ext_msgs, ob.n_ext_msgs, abi.MESSAGE),
                           (ob.results, ob.n_results, abi.CRESULT), (ob.ext_results, ob.n_ext_results, abi.RESULT)):
            a = np.zeros(n, dt)
            if n:
                ctypes.memmove(a.ctypes.data, ptr, n * dt.itemsize)
            out.append(a)
        _check(self.lib.gr_release_coutbox(self._h, ctypes.byref(ob)), "gr_release_coutbox")
        return tuple(out)

    def reserve_inbox(self, n_msgs, n_locals):
        """gr_inbox_reserve: (Inbox, msgs view, locals view) over engine-owned pinned
        memory; fill the views, then step_inbox(Inbox)."""
        ib = abi.Inbox()
        _check(self.lib.gr_inbox_reserve(self._h, n_msgs, n_locals, ctypes.byref(ib)), "gr_inbox_reserve")
        msgs = np.ctypeslib.as_array(ctypes.cast(ib.msgs, ctypes.POINTER(ctypes.c_uint8)),
                                     (max(n_msgs, 1) * abi.MESSAGE.itemsize,)).view(abi.MESSAGE)[:n_msgs]
        loc = np.ctypeslib.as_array(ctypes.cast(ib.locals, ctypes.POINTER(ctypes.c_uint8)),
                                    (max(n_locals, 1) * abi.LOCAL.itemsize,)).view(abi.LOCAL)[:n_locals]
        return ib, msgs, loc

    def stats(self):
        s = abi.Stats()
        _check(self.lib.gr_stats_get(self._h, ctypes.byref(s)), "gr_stats_get")
        return {k: getattr(s, k) for k, _ in abi.Stats._fields_}

    def reset_stats(self):
        _check(self.lib.gr_stats_reset(self._h), "gr_stats_reset")

    def timing_begin(self):
        """Record HIP events around each pass's two kernels until timing_end()."""
        _check(self.lib.gr_timing_begin(self._h), "gr_timing_begin")

    def timing_end(self):
        t = abi.Timing()
        _check(self.lib.gr_timing_end(self._h, ctypes.byref(t)), "gr_timing_end")
        return {k: getattr(t, k) for k, _ in abi.Timing._fields_}

    # ---- device-resident path -------------------------------------------------
    def space_bytes(self, n_chunks, positions, depth=MAILBOX_DEPTH):
        return int(self.lib.gr_space_bytes(n_chunks, positions, depth))

    def chunk_bytes(self, positions, depth=MAILBOX_DEPTH):
        return int(self.lib.gr_space_chunk_bytes(positions, depth))

    def hot_chunk_bytes(self, positions, depth=MAILBOX_DEPTH):
        return int(self.lib.gr_space_hot_chunk_bytes(positions, depth))

    def hot_tile_bytes(self, depth=MAILBOX_DEPTH):
        """Bytes per 64-position tile of a hot chunk (its first 64 are the count bytes)."""
        return int(self.lib.gr_space_hot_tile_bytes(depth))

    def cold_used(self, space_ptr, n_chunks, positions, depth=MAILBOX_DEPTH, stream=0):
        """True when some mailbox of the device space needs its cold fields (waits for `stream`)."""
        v = ctypes.c_uint32()
        _check(self.lib.gr_space_cold_used(self._h, space_ptr, n_chunks, positions, depth, stream,
                                           ctypes.byref(v)), "gr_space_cold_used")
        return bool(v.value)

    def side_bytes(self, n_chunks, depth, capacity):
        """Bytes of the side buffers of n_chunks chunks (gr_space_side_bytes)."""
        return int(self.lib.gr_space_side_bytes(n_chunks, depth, capacity))

    def side_pack(self, space_ptr, n_chunks, positions, depth, side_ptr, capacity, stream=0):
        """Compact the device space's cold fields into the side buffers, on `stream` (no wait)."""
        _check(self.lib.gr_space_side_pack(space_ptr, n_chunks, positions, depth, side_ptr, capacity, stream),
               "gr_space_side_pack")

    def side_unpack(self, space_ptr, n_chunks, positions, depth, side_ptr, capacity, stream=0):
        """Write received side-buffer entries into the device space's cold chunks, on `stream`."""
        _check(self.lib.gr_space_side_unpack(space_ptr, n_chunks, positions, depth, side_ptr, capacity, stream),
               "gr_space_side_unpack")

    def cx_bytes(self, n_chunks, positions, depth, capacities, side_capacity):
        """Bytes of the compact-exchange buffers of n_chunks chunks (gr_space_cx_bytes);
        capacities: the record capacity of each chunk."""
        caps = cx_caps_array(capacities, n_chunks)
        return int(self.lib.gr_space_cx_bytes(n_chunks, positions, depth, caps.ctypes.data, side_capacity))

    def cx_pack(self, space_ptr, n_chunks, positions, depth, cx_ptr, capacities, side_capacity, stream=0):
        """Pack the device out space's mailboxes into the compact buffers, on `stream` (no wait)."""
        caps = cx_caps_array(capacities, n_chunks)
        _check(self.lib.gr_space_cx_pack(space_ptr, n_chunks, positions, depth, cx_ptr, caps.ctypes.data,
                                         side_capacity, stream), "gr_space_cx_pack")

    def cx_unpack(self, space_ptr, n_chunks, positions, depth, cx_ptr, capacities, side_capacity, stream=0):
        """Write received compact buffers into the device in space, on `stream`."""
        caps = cx_caps_array(capacities, n_chunks)
        _check(self.lib.gr_space_cx_unpack(space_ptr, n_chunks, positions, depth, cx_ptr, caps.ctypes.data,
                                           side_capacity, stream), "gr_space_cx_unpack")

    def bind_routes(self, in_pos, out_pos):
        """in_pos/out_pos: uint32 arrays [slots][n_peers] (mailbox positions, 0xFFFFFFFF = none)."""
        in_pos = np.ascontiguousarray(in_pos, np.uint32)
        out_pos = np.ascontiguousarray(out_pos, np.uint32)
        n = in_pos.shape[1]
        _check(self.lib.gr_bind_routes(self._h, in_pos.ctypes.data, out_pos.ctypes.data, n), "gr_bind_routes")

    def set_locals(self, locals_):
        locals_ = np.ascontiguousarray(locals_, abi.LOCAL)
        _check(self.lib.gr_set_locals(self._h, locals_.ctypes.data if len(locals_) else None,
                                      len(locals_)), "gr_set_locals")

    def step_device(self, in_ptr, out_ptr, in_chunks, in_positions, out_chunks, out_positions,
                    n_peers, stream=0, depth=MAILBOX_DEPTH):
        _check(self.lib.gr_step_device(self._h, in_ptr, out_ptr, in_chunks, in_positions, out_chunks,
                                       out_positions, depth, n_peers, stream), "gr_step_device")

    def graph_capture(self, space_a, space_b, n_chunks, positions, n_peers, n_passes=2, depth=MAILBOX_DEPTH):
        """gr_graph_capture: n_passes (even) device passes over the ping-pong spaces
        (device pointers) recorded into a HIP graph; returns the graph handle."""
        g = ctypes.c_void_p()
        _check(self.lib.gr_graph_capture(self._h, space_a, space_b, n_chunks, positions, depth, n_peers, n_passes,
                                         ctypes.byref(g)), "gr_graph_capture")
        return g

    def graph_replay(self, g, stream=0):
        _check(self.lib.gr_graph_replay(g, stream), "gr_graph_replay")

    def graph_destroy(self, g):
        self.lib.gr_graph_destroy(g)

    def collect_results(self, n=None, first=0):
        n = self.max_peers - first if n is None else n
        out = np.zeros(n, abi.RESULT)
        _check(self.lib.gr_collect_results(self._h, first, out.ctypes.data, n), "gr_collect_results")
        return out


def cx_caps_array(capacities, n_chunks):
    """Per-chunk record capacities as the uint32 array the C-ABI takes (an int
    means the same capacity for every chunk)."""
    if np.isscalar(capacities):
        capacities = [capacities] * n_chunks
    caps = np.ascontiguousarray(capacities, np.uint32)
    assert len(caps) == n_chunks
    return caps


def decode_space(buf, n_chunks, positions, depth=MAILBOX_DEPTH, lost_ok=False):
    """Decode a host copy of a message space (bytes/uint8 array) into records.

    peer = mailbox position, slot = index within the mailbox. A mailbox whose
    cold fields were lost in the exchange decodes to records with reject 0xFF:
    an error unless lost_ok."""
    lib = load_library()
    buf = np.ascontiguousarray(buf, np.uint8)
    n = ctypes.c_size_t()
    _check(lib.gr_space_decode(buf.ctypes.data, n_chunks, positions, depth, None, 0, ctypes.byref(n)),
           "decode")
    out = np.zeros(n.value, abi.MESSAGE)
    if n.value:
        _check(lib.gr_space_decode(buf.ctypes.data, n_chunks, positions, depth, out.ctypes.data, n.value,
                                   ctypes.byref(n)), "decode")
    if not lost_ok and np.any(out["reject"] == 0xFF):
        raise RuntimeError("space holds mailboxes whose cold fields were lost in the exchange")
    return out
