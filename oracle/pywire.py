"""TEST INFRASTRUCTURE: ctypes bindings of the wire-codec oracle
(oracle/_build/liboraclewire.so, built from wire_oracle.hpp / wire_capi.cpp), a
seeded generator of raftpb records, and a minimal protobuf/colfer byte writer for
hand-built known-answer frames.

Only tests/, __graft_entry__.smoke() and tools/bench_wire.py's cpu_baseline leg
import this module. The product (dragonboat_amd) never does.
"""
import ctypes
import os

import numpy as np

from dragonboat_amd import wire as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_build", "liboraclewire.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        l = ctypes.CDLL(LIB)
        c = ctypes
        vp, sz, psz = c.c_void_p, c.c_size_t, c.POINTER(c.c_size_t)
        l.grwo_decode.argtypes = [vp, sz, vp, sz, vp, sz, vp, sz, psz, psz]
        l.grwo_encode.argtypes = [vp, sz, vp, sz, vp, sz, vp, sz, vp, sz, psz]
        l.grwo_decode_bench.argtypes = [vp, vp, sz, c.c_int, c.c_double, c.POINTER(c.c_uint64)]
        l.grwo_decode_bench.restype = c.c_double
        _lib = l
    return _lib


def _p(a):
    return a.ctypes.data if a is not None and a.size else None


def decode(buf, batches):
    """Oracle MessageBatch.Unmarshal of every frame; same contract as grw_decode."""
    buf = np.ascontiguousarray(np.frombuffer(bytes(buf), np.uint8) if not isinstance(buf, np.ndarray) else buf)
    nm, ne = ctypes.c_size_t(0), ctypes.c_size_t(0)
    msgs = np.zeros(0, W.WMESSAGE)
    ents = np.zeros(0, W.WENTRY)
    for _ in range(2):
        rc = lib().grwo_decode(_p(buf), buf.size, _p(batches), len(batches), _p(msgs), len(msgs), _p(ents),
                               len(ents), ctypes.byref(nm), ctypes.byref(ne))
        if rc == -5:
            msgs = np.zeros(nm.value, W.WMESSAGE)
            ents = np.zeros(ne.value, W.WENTRY)
            continue
        assert rc == 0, rc
        return batches, msgs[:nm.value], ents[:ne.value]
    raise AssertionError("oracle decode capacity")


def encode(payload, batches, msgs, ents):
    """Oracle MessageBatch.MarshalTo of every batch; returns the bytes."""
    payload = np.ascontiguousarray(payload, dtype=np.uint8)
    need = ctypes.c_size_t(0)
    out = np.zeros(0, np.uint8)
    for _ in range(2):
        rc = lib().grwo_encode(_p(payload), payload.size, _p(batches), len(batches), _p(msgs), len(msgs),
                               _p(ents), len(ents), _p(out), out.size, ctypes.byref(need))
        if rc == -5:
            out = np.zeros(need.value, np.uint8)
            continue
        assert rc == 0, rc
        return out[:need.value]
    raise AssertionError("oracle encode capacity")


def decode_bench(buf, batches, threads, seconds):
    reps = ctypes.c_uint64(0)
    rate = lib().grwo_decode_bench(_p(buf), _p(batches), len(batches), threads, seconds, ctypes.byref(reps))
    return rate, reps.value


# ----------------------------------------------------------- record generator --

def _mag(rng, n):
    """u64 values over every varint width, incl. 0, the colfer 2^49 switch and 2^64-1."""
    bits = rng.integers(0, 65, n)
    v = rng.integers(0, 2**63, n, dtype=np.uint64, endpoint=False) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    mask = np.where(bits >= 64, np.uint64(2**64 - 1), (np.uint64(1) << bits.astype(np.uint64)) - np.uint64(1))
    return v & mask


def make_records(n_batches, msgs_per_batch, seed, max_entries=3, cmd_len=16, steady=False, snap_frac=0.0):
    """Random raftpb records: batches, messages, entries and the payload they address.

    steady=True gives the step path's shapes (Replicate/ReplicateResp/Heartbeat with
    realistic magnitudes, 16-B Cmds); otherwise every field sweeps its full range."""
    rng = np.random.default_rng(seed)
    mpb = np.full(n_batches, msgs_per_batch) if np.isscalar(msgs_per_batch) else np.asarray(msgs_per_batch)
    nm = int(mpb.sum())
    b = np.zeros(n_batches, W.BATCH)
    b["n_msgs"] = mpb
    b["first_msg"] = np.concatenate([[0], np.cumsum(mpb)[:-1]]) if n_batches else []
    m = np.zeros(nm, W.WMESSAGE)
    if steady:
        base = np.uint64(2**32) + rng.integers(0, 2**20, nm).astype(np.uint64)
        m["type"] = rng.choice([12, 13, 17, 18], nm)
        m["to"] = rng.integers(1, 6, nm)
        m["from"] = rng.integers(1, 6, nm)
        m["cluster_id"] = rng.integers(1, 1 << 20, nm)
        m["term"] = rng.integers(1, 6, nm)
        m["log_term"] = m["term"]
        m["log_index"] = base
        m["commit"] = base - np.uint64(1)
        n_ent = np.where(m["type"] == 12, 1, 0)
    else:
        for f in ("to", "from", "cluster_id", "term", "log_term", "log_index", "commit", "hint", "hint_high"):
            m[f] = _mag(rng, nm)
        t = rng.integers(-2**31, 2**31, nm, dtype=np.int64)
        small = rng.random(nm) < 0.7
        t[small] = rng.integers(0, 25, int(small.sum()))
        m["type"] = t.astype(np.int32)
        m["reject"] = rng.integers(0, 2, nm)
        n_ent = rng.integers(0, max_entries + 1, nm)
    m["n_entries"] = n_ent
    m["first_entry"] = np.concatenate([[0], np.cumsum(n_ent)[:-1]]) if nm else []
    ne = int(n_ent.sum())
    e = np.zeros(ne, W.WENTRY)
    if steady:
        owner = np.repeat(np.arange(nm), n_ent)
        e["term"] = m["term"][owner]
        e["index"] = m["log_index"][owner] + np.uint64(1)
        e["key"] = rng.integers(0, 2**40, ne, dtype=np.uint64)
        e["client_id"] = rng.integers(0, 2**63, ne, dtype=np.uint64)
        e["series_id"] = rng.integers(0, 1000, ne, dtype=np.uint64)
        e["responded_to"] = np.maximum(e["series_id"].astype(np.int64) - 1, 0).astype(np.uint64)
        e["cmd_len"] = cmd_len
    else:
        for f in ("term", "index", "key", "client_id", "series_id", "responded_to"):
            e[f] = _mag(rng, ne)
            e[f][rng.random(ne) < 0.2] = 0
        e["type"] = np.where(rng.random(ne) < 0.2, rng.integers(-2**31, 2**31, ne, dtype=np.int64),
                             rng.integers(0, 4, ne)).astype(np.int32)
        e["cmd_len"] = np.where(rng.random(ne) < 0.2, 0, rng.integers(1, 300, ne))
    # payload: source addresses, cmds, a few non-zero snapshots
    src = [f"10.0.{rng.integers(0, 255)}.{rng.integers(0, 255)}:{rng.integers(1000, 65535)}".encode()
           for _ in range(n_batches)]
    cmd_total = int(e["cmd_len"].astype(np.int64).sum())
    snap_msgs = np.nonzero(rng.random(nm) < snap_frac)[0] if snap_frac else np.zeros(0, np.int64)
    snap_bytes = [bytes([0x12, 3]) + b"a/b" + bytes([0x20]) + _varint(int(rng.integers(1, 1 << 40)))
                  for _ in snap_msgs]
    total = sum(len(s) for s in src) + cmd_total + sum(len(s) for s in snap_bytes)
    payload = np.zeros(max(total, 1), np.uint8)
    off = 0
    for i, s in enumerate(src):
        payload[off:off + len(s)] = np.frombuffer(s, np.uint8)
        b["source_off"][i] = off
        b["source_len"][i] = len(s)
        off += len(s)
    if ne:
        lens = e["cmd_len"].astype(np.int64)
        e["cmd_off"] = off + np.concatenate([[0], np.cumsum(lens)[:-1]])
        payload[off:off + cmd_total] = rng.integers(0, 256, cmd_total, dtype=np.uint8)
        off += cmd_total
    for j, s in zip(snap_msgs, snap_bytes):
        payload[off:off + len(s)] = np.frombuffer(s, np.uint8)
        m["snapshot_off"][j] = off
        m["snapshot_len"][j] = len(s)
        off += len(s)
    b["deployment_id"] = rng.integers(0, 2**63, n_batches, dtype=np.uint64)
    b["bin_ver"] = rng.integers(0, 2**32, n_batches, dtype=np.uint64).astype(np.uint32)
    return payload, b, m, e


# ------------------------------------------------------- hand-built byte frames --

def _varint(v):
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def tag(field, wt):
    return _varint((field << 3) | wt)


def fld_varint(field, v):
    return tag(field, 0) + _varint(v)


def fld_bytes(field, data):
    return tag(field, 2) + _varint(len(data)) + bytes(data)


def colfer_entry(term=0, index=0, type_=0, key=0, client_id=0, series_id=0, responded_to=0, cmd=b""):
    """Entry.marshalTo (raft_optimized.go:160-295), written independently of the oracle."""
    out = bytearray()

    def u64f(h, x):
        if x >= 1 << 49:
            out.append(h | 0x80)
            out.extend(x.to_bytes(8, "big"))
        elif x:
            out.append(h)
            out.extend(_varint(x))

    u64f(0, term)
    u64f(1, index)
    if type_:
        x = type_ & 0xFFFFFFFF
        if type_ >= 0:
            out.append(2)
        else:
            x = (~x + 1) & 0xFFFFFFFF
            out.append(2 | 0x80)
        out.extend(_varint(x))
    u64f(3, key)
    u64f(4, client_id)
    u64f(5, series_id)
    u64f(6, responded_to)
    if cmd:
        out.append(7)
        out.extend(_varint(len(cmd)))
        out.extend(cmd)
    out.append(0x7F)
    return bytes(out)


ZERO_SNAPSHOT = bytes([0x12, 0x00, 0x18, 0x00, 0x20, 0x00, 0x28, 0x00, 0x32, 0x02, 0x08, 0x00])


def frames(*payloads):
    """Concatenate frames into one buffer; returns (buffer, grw_batch table)."""
    offs, lens, buf = [], [], bytearray()
    for p in payloads:
        offs.append(len(buf))
        lens.append(len(p))
        buf.extend(p)
    return np.frombuffer(bytes(buf) if buf else b"\0", np.uint8).copy(), W.frames_table(offs, lens)
