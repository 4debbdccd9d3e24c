"""Host side of the device wire codec (include/gpuraft_wire.h, libgrwire.so).

Mirrors the reference's raftpb codec entry points for a whole pass of frames:

- ``WireCodec.unmarshal`` = ``MessageBatch.Unmarshal`` (raftpb/raft_optimized.go:1050)
  applied to every frame a transport pass received (internal/transport/tcp.go:422);
- ``WireCodec.marshal`` = ``MessageBatch.MarshalTo`` (raftpb/raft.pb.go:1929) of every
  batch a send pass builds (internal/transport/transport.go:399-470).

Records are numpy structured arrays with the C layouts; byte payloads (Entry.Cmd,
SourceAddress) stay in the frame buffer and are addressed by offset. Errors follow
the reference: a frame Go would reject carries its status (``STATUS_NAMES``), and the
call itself only fails (``WireError``) for bad arguments or a device failure. There is
no CPU fallback: without libgrwire.so or a GPU the codec refuses to run.
"""
import ctypes
import os

import numpy as np

from dragonboat_amd.abi import u8, u32, u64

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "dragonboat_amd", "_build", "libgrwire.so")

i32 = np.int32

OK, E_INT_OVERFLOW, E_UNEXPECTED_EOF, E_INVALID_LENGTH, E_END_GROUP, E_ILLEGAL_TAG = range(6)
E_WRONG_WIRE_TYPE, E_ILLEGAL_WIRE_TYPE, E_ENTRY_EOF, E_ENTRY_HEADER, E_ENTRY_MAX, E_PANIC = range(6, 12)
STATUS_NAMES = ["ok", "ErrIntOverflowRaft", "io.ErrUnexpectedEOF", "ErrInvalidLengthRaft",
                "wiretype end group for non-group", "illegal tag", "wrong wireType", "illegal wireType",
                "colfer io.EOF", "ColferError", "ColferMax", "panic"]
LVL_BATCH, LVL_MESSAGE, LVL_ENTRY = 0, 1, 2
COLFER_SIZE_MAX = 256 * 1024 * 1024

BATCH = np.dtype([
    ("deployment_id", u64), ("frame_off", u64), ("source_off", u64), ("frame_len", u32),
    ("source_len", u32), ("first_msg", u32), ("n_msgs", u32), ("bin_ver", u32), ("status", i32),
    ("err_msg", u32), ("err_field", u32), ("err_level", u8), ("pad", u8, (7,)),
])
WMESSAGE = np.dtype([
    ("to", u64), ("from", u64), ("cluster_id", u64), ("term", u64), ("log_term", u64),
    ("log_index", u64), ("commit", u64), ("hint", u64), ("hint_high", u64), ("msg_off", u64),
    ("snapshot_off", u64), ("msg_len", u32), ("snapshot_len", u32), ("first_entry", u32),
    ("n_entries", u32), ("batch", u32), ("type", i32), ("reject", u8), ("snapshot_host", u8),
    ("pad", u8, (6,)),
])
WENTRY = np.dtype([
    ("term", u64), ("index", u64), ("key", u64), ("client_id", u64), ("series_id", u64),
    ("responded_to", u64), ("cmd_off", u64), ("cmd_len", u32), ("type", i32),
])
assert BATCH.itemsize == 64 and WMESSAGE.itemsize == 120 and WENTRY.itemsize == 64

# Every symbol include/gpuraft_wire.h declares.
EXPORTS = ["grw_create", "grw_destroy", "grw_status_name", "grw_decode", "grw_decode_device",
           "grw_encode", "grw_encode_device", "grw_last_timing"]

# Message fields compared for parity (the values the Go struct holds).
MSG_VALUE_FIELDS = ["to", "from", "cluster_id", "term", "log_term", "log_index", "commit", "hint",
                    "hint_high", "type", "reject", "snapshot_host", "n_entries", "msg_off", "msg_len"]
ENTRY_FIELDS = list(WENTRY.names)
BATCH_VALUE_FIELDS = ["deployment_id", "source_off", "source_len", "bin_ver", "n_msgs", "status"]
BATCH_ERR_FIELDS = ["status", "err_level", "err_msg", "err_field", "n_msgs"]


class WireError(RuntimeError):
    pass


class Timing(ctypes.Structure):
    _fields_ = [("walk_ms", ctypes.c_float), ("scan_ms", ctypes.c_float), ("message_ms", ctypes.c_float),
                ("entry_ms", ctypes.c_float), ("total_ms", ctypes.c_float)]


def load_library(path=LIB_PATH):
    if not os.path.exists(path):
        raise WireError(f"{path} is not built: run __graft_entry__.build() (no CPU fallback exists)")
    lib = ctypes.CDLL(path)
    c = ctypes
    lib.grw_create.argtypes = [c.c_uint32, c.POINTER(c.c_void_p)]
    lib.grw_destroy.argtypes = [c.c_void_p]
    lib.grw_destroy.restype = None
    lib.grw_status_name.restype = c.c_char_p
    sz = c.c_size_t
    psz = c.POINTER(c.c_size_t)
    vp = c.c_void_p
    lib.grw_decode.argtypes = [vp, vp, sz, vp, sz, vp, sz, vp, sz, psz, psz]
    lib.grw_decode_device.argtypes = [vp, vp, sz, vp, sz, vp, sz, vp, sz, psz, psz]
    lib.grw_encode.argtypes = [vp, vp, sz, vp, sz, vp, sz, vp, sz, vp, sz, psz]
    lib.grw_encode_device.argtypes = [vp, vp, sz, vp, sz, vp, sz, vp, sz, vp, sz, psz]
    lib.grw_last_timing.argtypes = [vp, c.POINTER(Timing)]
    return lib


def _ptr(a):
    return a.ctypes.data if a is not None and a.size else None


def frames_table(offsets, lengths):
    """grw_batch records naming frames (offset, length) of one buffer."""
    b = np.zeros(len(offsets), BATCH)
    b["frame_off"] = offsets
    b["frame_len"] = lengths
    return b


class WireCodec:
    """One device codec context (one HIP stream) for the wire passes of a transport."""

    def __init__(self, device=0):
        self.lib = load_library()
        h = ctypes.c_void_p()
        rc = self.lib.grw_create(device, ctypes.byref(h))
        if rc != 0:
            raise WireError(f"grw_create failed ({rc}): no usable GPU")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.grw_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def unmarshal(self, buf, batches):
        """MessageBatch.Unmarshal of every frame ``batches`` names in ``buf`` (host arrays).

        Returns (batches, messages, entries); batches are updated in place."""
        buf = np.ascontiguousarray(np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else buf)
        nm, ne = ctypes.c_size_t(0), ctypes.c_size_t(0)
        msgs = np.zeros(0, WMESSAGE)
        ents = np.zeros(0, WENTRY)
        for _ in range(3):  # capacity: the message total, then the entry total, come back first
            rc = self.lib.grw_decode(self.h, _ptr(buf), buf.size, _ptr(batches), len(batches), _ptr(msgs),
                                     len(msgs), _ptr(ents), len(ents), ctypes.byref(nm), ctypes.byref(ne))
            if rc == -5:
                if nm.value > len(msgs):
                    msgs = np.zeros(nm.value, WMESSAGE)
                if ne.value > len(ents):
                    ents = np.zeros(ne.value, WENTRY)
                continue
            if rc != 0:
                raise WireError(f"grw_decode failed ({rc})")
            return batches, msgs[:nm.value], ents[:ne.value]
        raise WireError("grw_decode: totals changed between calls")

    def marshal(self, payload, batches, msgs, ents):
        """MessageBatch.MarshalTo of every batch; returns the frames' bytes (frame_off/frame_len set)."""
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        need = ctypes.c_size_t(0)
        out = np.zeros(0, np.uint8)
        for _ in range(2):
            rc = self.lib.grw_encode(self.h, _ptr(payload), payload.size, _ptr(batches), len(batches),
                                     _ptr(msgs), len(msgs), _ptr(ents), len(ents), _ptr(out), out.size,
                                     ctypes.byref(need))
            if rc == -5:
                out = np.zeros(need.value, np.uint8)
                continue
            if rc != 0:
                raise WireError(f"grw_encode failed ({rc})")
            return out[:need.value]
        raise WireError("grw_encode: output size changed between calls")

    def unmarshal_device(self, d_buf, buf_len, d_batches, n, d_msgs, msg_cap, d_ents, ent_cap, stream_sync=True):
        """grw_decode_device over device pointers (ints); returns (n_msgs, n_ents)."""
        nm, ne = ctypes.c_size_t(0), ctypes.c_size_t(0)
        rc = self.lib.grw_decode_device(self.h, d_buf, buf_len, d_batches, n, d_msgs, msg_cap, d_ents, ent_cap,
                                        ctypes.byref(nm), ctypes.byref(ne))
        if rc != 0:
            raise WireError(f"grw_decode_device failed ({rc}); totals {nm.value} msgs, {ne.value} entries")
        return nm.value, ne.value

    def marshal_device(self, d_payload, payload_len, d_batches, n, d_msgs, n_msgs, d_ents, n_ents, d_out, out_cap):
        need = ctypes.c_size_t(0)
        rc = self.lib.grw_encode_device(self.h, d_payload, payload_len, d_batches, n, d_msgs, n_msgs, d_ents,
                                        n_ents, d_out, out_cap, ctypes.byref(need))
        if rc != 0:
            raise WireError(f"grw_encode_device failed ({rc}); needs {need.value} bytes")
        return need.value

    def timing(self):
        t = Timing()
        self.lib.grw_last_timing(self.h, ctypes.byref(t))
        return {k: getattr(t, k) for k, _ in Timing._fields_}
