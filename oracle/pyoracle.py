"""TEST INFRASTRUCTURE: ctypes bindings of the oracle (oracle/_build/liboracle.so)
and of the test-only host-lane harness (tests/_build/libhostlane.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module. The product (dragonboat_amd) never does.
"""
import ctypes
import os

import numpy as np

from dragonboat_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# GR_ORACLE_LIB / GR_HOSTLANE_LIB: another build of the same code (the
# sanitizer builds of tests/test_sanitizers.py)
ORACLE_LIB = os.environ.get("GR_ORACLE_LIB") or os.path.join(ROOT, "oracle", "_build", "liboracle.so")
HOSTLANE_LIB = os.environ.get("GR_HOSTLANE_LIB") or os.path.join(ROOT, "tests", "_build", "libhostlane.so")
KAT_BIN = os.path.join(ROOT, "oracle", "_build", "kat_tests")

_olib = None
_hlib = None


def oracle_lib():
    global _olib
    if _olib is None:
        lib = ctypes.CDLL(ORACLE_LIB)
        c = ctypes
        lib.ob_create.argtypes = [c.c_uint32, c.c_uint64, c.c_void_p, c.c_uint32, c.POINTER(c.c_void_p)]
        lib.ob_destroy.argtypes = [c.c_void_p]
        lib.ob_destroy.restype = None
        lib.ob_export.argtypes = [c.c_void_p, c.c_void_p, c.c_uint32]
        lib.ob_commit_all.argtypes = [c.c_void_p]
        lib.ob_commit_all_mt.argtypes = [c.c_void_p, c.c_uint32]
        lib.ob_rehome.argtypes = [c.c_void_p, c.c_uint32]
        lib.ob_representable.argtypes = [c.c_void_p, c.c_void_p, c.c_uint32]
        lib.ob_reload.argtypes = [c.c_void_p, c.c_uint32, c.c_void_p]
        lib.ob_step.argtypes = [c.c_void_p, c.POINTER(abi.Inbox), c.c_void_p, c.c_void_p, c.c_void_p,
                                c.c_void_p, c.c_size_t, c.POINTER(c.c_size_t), c.c_void_p, c.c_uint32,
                                c.c_char_p, c.c_size_t]
        lib.ob_step2.argtypes = [c.c_void_p, c.POINTER(abi.Inbox), c.c_void_p, c.c_void_p, c.c_uint32, c.c_uint32,
                                 c.c_uint32, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t,
                                 c.POINTER(c.c_size_t), c.c_void_p, c.c_uint32, c.c_char_p, c.c_size_t]
        lib.ob_fetch_out.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t]
        lib.ob_set_truncate_runs.argtypes = [c.c_void_p, c.c_int]
        lib.ob_commit_update.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_uint32, c.c_void_p]
        _olib = lib
    return _olib


def hostlane_lib():
    global _hlib
    if _hlib is None:
        lib = ctypes.CDLL(HOSTLANE_LIB)
        c = ctypes
        lib.hl_step.argtypes = [c.c_uint32, c.c_uint64, c.c_void_p, c.c_uint32, c.POINTER(abi.Inbox),
                                c.c_void_p, c.c_size_t, c.POINTER(c.c_size_t), c.c_void_p,
                                c.POINTER(c.c_size_t)]
        lib.hl_commit_update.argtypes = [c.c_uint32, c.c_void_p, c.c_uint32, c.c_void_p, c.c_void_p, c.c_uint32,
                                         c.c_void_p]
        lib.hl_counters.argtypes = [c.POINTER(c.c_uint64), c.POINTER(c.c_uint64)]
        lib.hl_counters.restype = None
        lib.hl_tick_lanes.restype = c.c_uint64
        lib.hl_steady_lanes.restype = c.c_uint64
        lib.hl_steady_leaders.restype = c.c_uint64
        lib.hl_detect_affine.argtypes = [c.c_void_p, c.c_void_p, c.c_uint32, c.c_uint32, c.c_void_p,
                                         c.POINTER(c.c_uint32)]
        lib.hl_detect_affine.restype = c.c_int
        _hlib = lib
    return _hlib


class OracleError(RuntimeError):
    pass


class OraclePopulation:
    """Faithful per-group raft objects (the CPU restatement of internal/raft)."""

    def __init__(self, peers, slots=3, max_entry_size=abi.MAX_ENTRY_SIZE):
        self.lib = oracle_lib()
        peers = np.ascontiguousarray(peers, abi.PEER)
        h = ctypes.c_void_p()
        rc = self.lib.ob_create(slots, max_entry_size, peers.ctypes.data, len(peers), ctypes.byref(h))
        if rc:
            raise OracleError(f"ob_create failed {rc}")
        self._h = h
        self.n = len(peers)
        self.slots = slots

    def __del__(self):
        if getattr(self, "_h", None):
            self.lib.ob_destroy(self._h)
            self._h = None

    def set_truncate_runs(self, on=True):
        """CPU-baseline mode: Replicates spanning more than 2 term runs travel with
        their first two runs (a prefix of the entries, as a size-limited send);
        parity runs leave this off and such a message is an error."""
        self.lib.ob_set_truncate_runs(self._h, 1 if on else 0)

    def commit_update(self, slots, uc):
        """entryLog.commitUpdate per slot (ob_commit_update): (rc, status)."""
        slots = np.ascontiguousarray(slots, np.uint32)
        uc = np.ascontiguousarray(uc, abi.UPDATE_COMMIT)
        st = np.zeros(len(slots), np.int32)
        rc = self.lib.ob_commit_update(self._h, slots.ctypes.data if len(slots) else None,
                                       uc.ctypes.data if len(uc) else None, len(slots),
                                       st.ctypes.data if len(st) else None)
        return rc, st

    def export(self):
        out = np.zeros(self.n, abi.PEER)
        self.lib.ob_export(self._h, out.ctypes.data, self.n)
        return out

    def representable(self):
        """bool[n]: the peer's state fits a gr_peer record (device-resident)."""
        out = np.zeros(self.n, np.uint8)
        self.lib.ob_representable(self._h, out.ctypes.data, self.n)
        return out.astype(bool)

    def reload(self, idx, recs):
        """Rebuild peers from records (state injections)."""
        for p, rec in zip(idx, recs):
            r = np.array([rec], abi.PEER)
            rc = self.lib.ob_reload(self._h, int(p), r.ctypes.data)
            if rc:
                raise OracleError(f"ob_reload failed {rc}")

    def commit_all(self, threads=1):
        """Persist + apply everything (threads > 1: on the step's worker partition)."""
        if threads > 1:
            self.lib.ob_commit_all_mt(self._h, threads)
        else:
            self.lib.ob_commit_all(self._h)

    def rehome(self, threads):
        """Rebuild each peer on the worker thread that steps it (CPU baseline)."""
        if self.lib.ob_rehome(self._h, threads):
            raise OracleError("ob_rehome failed")

    def step(self, msgs=None, locals_=None, limits=None, threads=1, allow_error=False, dev_before=None,
             in_depth=abi.GR_C, out_depth=abi.GR_C, has_locals=True, want_mid=True):
        """Returns dict(msgs, items, results, mid, error, esc_mask).

        esc_mask[p] (when limits are given) is the set of gr_escalation reasons,
        bit r, that the oracle's own execution of item limits[p] justifies: the
        escalation predicate (batch.cpp). dev_before = device state at the start
        of the pass (its term-run window is modelled); None uses the oracle's."""
        msgs = np.zeros(0, abi.MESSAGE) if msgs is None else np.ascontiguousarray(msgs, abi.MESSAGE)
        locals_ = np.zeros(0, abi.LOCAL) if locals_ is None else np.ascontiguousarray(locals_, abi.LOCAL)
        ib = abi.inbox_of(msgs, locals_)
        lim = None
        if limits is not None:
            lim = np.ascontiguousarray(limits, np.uint32)
        db = None
        if dev_before is not None:
            db = np.ascontiguousarray(dev_before, abi.PEER)
            assert len(db) == self.n
        mid = np.zeros(self.n, abi.PEER) if want_mid else None  # want_mid=False: no per-peer export
        res = np.zeros(self.n, abi.RESULT)
        mask = np.zeros(self.n, np.uint32)
        n_out = ctypes.c_size_t()
        err = ctypes.create_string_buffer(512)
        rc = self.lib.ob_step2(self._h, ctypes.byref(ib), lim.ctypes.data if lim is not None else None,
                               db.ctypes.data if db is not None else None, in_depth, out_depth,
                               1 if has_locals else 0, mask.ctypes.data, mid.ctypes.data if want_mid else None,
                               None, None, 0, ctypes.byref(n_out), res.ctypes.data, threads, err, 512)
        n = n_out.value
        out = np.empty(n, abi.MESSAGE)  # sized exactly: the library kept the messages
        items = np.empty(n, np.uint32)
        rc2 = self.lib.ob_fetch_out(self._h, out.ctypes.data if n else None, items.ctypes.data if n else None, n)
        if rc2:
            raise OracleError(f"ob_fetch_out rc={rc2}")
        if rc and not (allow_error and rc == -6):
            raise OracleError(f"ob_step rc={rc}: {err.value.decode()}")
        return {"msgs": out, "items": items, "results": res, "mid": mid,
                "error": err.value.decode() if rc else "", "esc_mask": mask}


def hostlane_step(peers, msgs=None, locals_=None, slots=3, max_entry_size=abi.MAX_ENTRY_SIZE):
    """Run the engine's lane code on the CPU (test-only). Returns (peers', msgs, results)."""
    lib = hostlane_lib()
    peers = np.array(peers, dtype=abi.PEER, copy=True)
    msgs = np.zeros(0, abi.MESSAGE) if msgs is None else np.ascontiguousarray(msgs, abi.MESSAGE)
    locals_ = np.zeros(0, abi.LOCAL) if locals_ is None else np.ascontiguousarray(locals_, abi.LOCAL)
    ib = abi.inbox_of(msgs, locals_)
    cap = max(16, 8 * len(peers) * slots)
    out = np.zeros(cap, abi.MESSAGE)
    n_out = ctypes.c_size_t()
    res = np.zeros(len(peers), abi.RESULT)
    n_res = ctypes.c_size_t()
    rc = lib.hl_step(slots, max_entry_size, peers.ctypes.data, len(peers), ctypes.byref(ib), out.ctypes.data,
                     cap, ctypes.byref(n_out), res.ctypes.data, ctypes.byref(n_res))
    if rc:
        raise OracleError(f"hl_step rc={rc}")
    return peers, out[:n_out.value], res[:n_res.value]


def hostlane_counters():
    """(lanes finished by the lean steady-state lane, lanes it handed to the general lane)."""
    lib = hostlane_lib()
    f, b = ctypes.c_uint64(), ctypes.c_uint64()
    lib.hl_counters(ctypes.byref(f), ctypes.byref(b))
    return f.value, b.value


def hostlane_tick_lanes():
    """Lanes the heartbeat/ReadIndex/tick lane (gr_tick.h) finished since load."""
    return int(hostlane_lib().hl_tick_lanes())



def hostlane_steady_lanes():
    """Lanes the emulated steady kernel (gr_steady.h closed forms) finished since load."""
    return int(hostlane_lib().hl_steady_lanes())


def hostlane_steady_leaders():
    """Leader lanes the emulated steady kernel's SteadyLeader finished since load."""
    return int(hostlane_lib().hl_steady_leaders())


def hostlane_affine_routes(in_pos, out_pos, slots):
    """gr_bind_routes' route detection (test-only host build): (base [2][8][8], G, mode) or None."""
    lib = hostlane_lib()
    in_pos = np.ascontiguousarray(in_pos, np.uint32)
    out_pos = np.ascontiguousarray(out_pos, np.uint32)
    base = np.zeros((2, abi.GR_SMAX, abi.GR_SMAX), np.uint32)
    g = ctypes.c_uint32()
    mode = lib.hl_detect_affine(in_pos.ctypes.data, out_pos.ctypes.data, in_pos.shape[1], slots,
                                base.ctypes.data, ctypes.byref(g))
    return (base, g.value, "loopback" if mode == 2 else "affine") if mode else None


def hostlane_commit_update(peers, idx, uc, slots=3):
    """gr_commit_update on records with the engine's commit_marks (test-only).
    Edits `peers` in place; returns (rc, status)."""
    lib = hostlane_lib()
    idx = np.ascontiguousarray(idx, np.uint32)
    uc = np.ascontiguousarray(uc, abi.UPDATE_COMMIT)
    st = np.zeros(len(idx), np.int32)
    assert peers.flags["C_CONTIGUOUS"] and peers.dtype == abi.PEER
    rc = lib.hl_commit_update(slots, peers.ctypes.data, len(peers), idx.ctypes.data if len(idx) else None,
                              uc.ctypes.data if len(uc) else None, len(idx), st.ctypes.data if len(st) else None)
    return rc, st
