"""Wire codec: MessageBatch/Message/Entry unmarshal and marshal.

CPU tests pin the oracle (oracle/wire_oracle.hpp) against known-answer byte frames
built independently here (protobuf varints, colfer entries, every Go error path) and
against the reference's own raftpb tests (raftpb/raft_test.go:211-353); -m gpu tests
compare libgrwire.so with the oracle on the same inputs, bit for bit.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from dragonboat_amd import wire as W
from oracle import pywire as PW

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAX64 = 2**64 - 1


@pytest.fixture(scope="module")
def wbuilt():
    from dragonboat_amd import build
    build.build_wire_oracle()
    build.build_wire()
    return True


def dec1(*frames):
    buf, b = PW.frames(*frames)
    return PW.decode(buf, b)


def msg(*fields):
    return b"".join(fields)


def in_batch(*messages, tail=b""):
    return b"".join(PW.fld_bytes(1, m) for m in messages) + tail


# ------------------------------------------------------------ header / ABI --

def test_header_declares_exactly_the_exports():
    src = open(os.path.join(ROOT, "include", "gpuraft_wire.h")).read()
    decl = sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(grw_\w+)\(", src, re.M)))
    assert decl == sorted(W.EXPORTS)


def test_library_loads_and_exports(wbuilt):
    lib = ctypes.CDLL(W.LIB_PATH)
    assert not [s for s in W.EXPORTS if not hasattr(lib, s)]
    lib.grw_status_name.restype = ctypes.c_char_p
    assert lib.grw_status_name(W.E_PANIC) == b"panic"
    assert lib.grw_status_name(W.E_UNEXPECTED_EOF) == b"io.ErrUnexpectedEOF"


# ---------------------------------------------------------- known answers ---

def test_zero_message_bytes(wbuilt):
    # Message{}.MarshalTo (raft.pb.go:1747-1809): every scalar field is written,
    # Reject as one byte, the zero Snapshot as its 12 canonical bytes.
    b = np.zeros(1, W.BATCH)
    b["n_msgs"] = 1
    m = np.zeros(1, W.WMESSAGE)
    out = PW.encode(np.zeros(1, np.uint8), b, m, np.zeros(0, W.WENTRY)).tobytes()
    body = bytes([0x08, 0, 0x10, 0, 0x18, 0, 0x20, 0, 0x28, 0, 0x30, 0, 0x38, 0, 0x40, 0, 0x48, 0, 0x50, 0,
                  0x62, 12]) + PW.ZERO_SNAPSHOT + bytes([0x68, 0])
    assert out == bytes([0x0a, len(body)]) + body + bytes([0x10, 0, 0x1a, 0, 0x20, 0])
    assert int(b["frame_len"][0]) == len(out)


def test_varint_known_answers(wbuilt):
    # protobuf base-128 varints: 300 -> ac 02; 2^64-1 -> 9 x ff + 01
    b = np.zeros(1, W.BATCH)
    b["n_msgs"] = 1
    m = np.zeros(1, W.WMESSAGE)
    m["term"] = 300
    m["hint"] = MAX64
    m["type"] = -1  # int32 -1 is written as uint64(-1): ten bytes
    out = PW.encode(np.zeros(1, np.uint8), b, m, np.zeros(0, W.WENTRY)).tobytes()
    assert bytes([0x28, 0xac, 0x02]) in out
    assert bytes([0x50]) + b"\xff" * 9 + b"\x01" in out
    assert bytes([0x08]) + b"\xff" * 9 + b"\x01" in out
    bb, mm, _ = dec1(out)
    assert bb["status"][0] == W.OK and int(mm["term"][0]) == 300 and int(mm["hint"][0]) == MAX64
    assert int(mm["type"][0]) == -1


@pytest.mark.parametrize("ent", [
    dict(term=1, index=2, cmd=b"ab"),
    dict(term=2**49, index=2**49 - 1),  # the colfer fixed-width switch
    dict(term=MAX64, index=MAX64, type_=1, key=MAX64, client_id=MAX64, series_id=MAX64, responded_to=MAX64,
         cmd=bytes(range(200))),
    dict(type_=-1), dict(type_=-(2**31)), dict(type_=2**31 - 1),
    dict(),
])
def test_colfer_entry_known_answers(wbuilt, ent):
    """Entry.marshalTo (raft_optimized.go:160-295) restated independently in pywire
    equals the oracle's bytes, and decodes back to the same values."""
    cmd = ent.get("cmd", b"")
    payload = np.frombuffer(cmd + b"\0", np.uint8).copy()
    e = np.zeros(1, W.WENTRY)
    for k, f in [("term", "term"), ("index", "index"), ("key", "key"), ("client_id", "client_id"),
                 ("series_id", "series_id"), ("responded_to", "responded_to")]:
        e[f] = ent.get(k, 0)
    e["type"] = ent.get("type_", 0)
    e["cmd_len"] = len(cmd)
    m = np.zeros(1, W.WMESSAGE)
    m["n_entries"] = 1
    b = np.zeros(1, W.BATCH)
    b["n_msgs"] = 1
    out = PW.encode(payload, b, m, e).tobytes()
    want = PW.colfer_entry(**ent)
    assert bytes([0x5a]) + PW._varint(len(want)) + want in out
    bb, mm, ee = dec1(out)
    assert bb["status"][0] == W.OK and len(ee) == 1
    for f in ("term", "index", "key", "client_id", "series_id", "responded_to", "type", "cmd_len"):
        assert ee[f][0] == e[f][0], f
    if cmd:
        assert out[int(ee["cmd_off"][0]):int(ee["cmd_off"][0]) + len(cmd)] == cmd


# (frame bytes, status, level, err_msg, err_field) — every error the Go decoders return
M0 = msg(PW.fld_varint(1, 12), PW.fld_varint(5, 3))  # a valid Message
ERROR_CASES = {
    "truncated_tag": (b"\x80", W.E_UNEXPECTED_EOF, W.LVL_BATCH, 0, 0),
    "int_overflow": (b"\xff" * 10 + b"\x01", W.E_INT_OVERFLOW, W.LVL_BATCH, 0, 0),
    "end_group": (PW.tag(1, 4), W.E_END_GROUP, W.LVL_BATCH, 0, 0),
    "illegal_tag_zero": (b"\x00", W.E_ILLEGAL_TAG, W.LVL_BATCH, 0, 0),
    "illegal_tag_negative": (PW._varint((0x80000000 << 3) | 0) + b"\x00", W.E_ILLEGAL_TAG, W.LVL_BATCH, 0,
                             0x80000000),
    "wrong_wire_type_requests": (PW.fld_varint(1, 5), W.E_WRONG_WIRE_TYPE, W.LVL_BATCH, 0, 1),
    "wrong_wire_type_binver": (PW.fld_bytes(1, M0) + PW.fld_bytes(4, b"x"), W.E_WRONG_WIRE_TYPE, W.LVL_BATCH,
                               1, 4),
    "invalid_length": (PW.tag(1, 2) + PW._varint(1 << 63), W.E_INVALID_LENGTH, W.LVL_BATCH, 0, 0),
    "message_past_end": (PW.tag(1, 2) + b"\x05\x08", W.E_UNEXPECTED_EOF, W.LVL_BATCH, 0, 0),
    "source_past_end": (PW.tag(3, 2) + b"\x09abc", W.E_UNEXPECTED_EOF, W.LVL_BATCH, 0, 0),
    # messageCount (raft_optimized.go:1014) indexes past the slice: a Go panic at message 0
    "message_count_panic": (PW.fld_bytes(1, M0) + PW.tag(1, 2) + b"\x80", W.E_PANIC, W.LVL_BATCH, 0, 0),
    # ... but stops at the first non-Requests field, so the walk's own error stands
    "message_count_stops": (PW.fld_bytes(1, M0) + PW.fld_varint(2, 1) + PW.tag(1, 2) + b"\x80",
                            W.E_UNEXPECTED_EOF, W.LVL_BATCH, 1, 0),
    "slice_overflow_panic": (PW.fld_bytes(1, M0) + PW.tag(3, 2) + PW._varint((1 << 63) - 2), W.E_PANIC,
                             W.LVL_BATCH, 1, 0),
    "msg_wrong_wire_type": (in_batch(msg(PW.fld_bytes(5, b"x"))), W.E_WRONG_WIRE_TYPE, W.LVL_MESSAGE, 0, 5),
    "msg_end_group": (in_batch(M0, msg(PW.tag(7, 4))), W.E_END_GROUP, W.LVL_MESSAGE, 1, 0),
    "msg_truncated_varint": (in_batch(M0, M0, msg(PW.tag(6, 0) + b"\x80")), W.E_UNEXPECTED_EOF,
                             W.LVL_MESSAGE, 2, 0),
    "msg_int_overflow": (in_batch(msg(PW.tag(2, 0) + b"\x80" * 10 + b"\x01")), W.E_INT_OVERFLOW,
                         W.LVL_MESSAGE, 0, 0),
    "msg_illegal_wire_type": (in_batch(msg(PW.tag(20, 6))), W.E_ILLEGAL_WIRE_TYPE, W.LVL_MESSAGE, 0, 0),
    "msg_unclosed_group": (in_batch(msg(PW.tag(20, 3) + PW.fld_varint(1, 1))), W.E_UNEXPECTED_EOF,
                           W.LVL_MESSAGE, 0, 0),
    # entryCount (raft_optimized.go:979) runs off the message: panic
    "entry_count_panic": (in_batch(msg(PW.fld_bytes(11, PW.colfer_entry(term=1)), PW.tag(11, 2) + b"\x80")),
                          W.E_PANIC, W.LVL_MESSAGE, 0, 0),
    "entry_eof_empty": (in_batch(msg(PW.fld_bytes(11, b""))), W.E_ENTRY_EOF, W.LVL_ENTRY, 0, 0),
    "entry_eof_short": (in_batch(msg(PW.fld_bytes(11, b"\x00\x01"))), W.E_ENTRY_EOF, W.LVL_ENTRY, 0, 0),
    "entry_bad_header": (in_batch(M0, msg(PW.fld_bytes(11, b"\x09\x7f"))), W.E_ENTRY_HEADER, W.LVL_ENTRY, 1, 0),
    "entry_fields_out_of_order": (in_batch(msg(PW.fld_bytes(11, b"\x03\x05\x00\x01\x7f"))), W.E_ENTRY_HEADER,
                                  W.LVL_ENTRY, 0, 0),
    "entry_cmd_too_big": (in_batch(msg(PW.fld_bytes(11, b"\x07" + PW._varint(2**28 + 1) + b"\x7f"))),
                          W.E_ENTRY_MAX, W.LVL_ENTRY, 0, 0),
    "entry_cmd_short": (in_batch(msg(PW.fld_bytes(11, b"\x07\x05ab\x7f"))), W.E_ENTRY_EOF, W.LVL_ENTRY, 0, 0),
    "entry_type_short": (in_batch(msg(PW.fld_bytes(11, b"\x02\x01"))), W.E_ENTRY_EOF, W.LVL_ENTRY, 0, 0),
    "snapshot_wrong_wire_type": (in_batch(msg(PW.fld_varint(12, 0))), W.E_WRONG_WIRE_TYPE, W.LVL_MESSAGE, 0,
                                 12),
}


@pytest.mark.parametrize("name", sorted(ERROR_CASES))
def test_error_known_answers(wbuilt, name):
    frame, st, lvl, at, field = ERROR_CASES[name]
    bb, _, _ = dec1(frame)
    got = (int(bb["status"][0]), int(bb["err_level"][0]), int(bb["err_msg"][0]), int(bb["err_field"][0]))
    assert got == (st, lvl, at, field), (name, got)


def test_unknown_fields_are_skipped(wbuilt):
    """skipRaft (raft.pb.go:5139): varint, fixed64, bytes, nested groups, fixed32."""
    unknown = (PW.fld_varint(14, 7) + PW.tag(15, 1) + b"12345678" + PW.fld_bytes(16, b"xyz") +
               PW.tag(17, 3) + PW.fld_varint(1, 1) + PW.tag(18, 3) + PW.tag(18, 4) + PW.tag(17, 4) +
               PW.tag(19, 5) + b"1234")
    m = msg(PW.fld_varint(1, 13), unknown, PW.fld_varint(5, 9), PW.fld_varint(5, 11),  # last wins
            PW.fld_varint(9, 2), PW.fld_varint(1, (1 << 33) | 12))  # Reject 2 -> true, Type low 32 bits
    frame = in_batch(m, tail=unknown + PW.fld_varint(2, 77) + PW.fld_varint(4, (1 << 32) | 5) +
                     PW.fld_bytes(3, b"host:1"))
    bb, mm, _ = dec1(frame)
    assert bb["status"][0] == W.OK and bb["n_msgs"][0] == 1
    assert int(bb["deployment_id"][0]) == 77 and int(bb["bin_ver"][0]) == 5
    assert int(bb["source_len"][0]) == 6
    assert int(mm["term"][0]) == 11 and mm["reject"][0] == 1 and int(mm["type"][0]) == 12


def test_snapshot_classification(wbuilt):
    cases = [(b"", 0), (PW.ZERO_SNAPSHOT, 0), (PW.fld_varint(4, 9), 1), (PW.ZERO_SNAPSHOT[:-2], 1)]
    for snap, host in cases:
        bb, mm, _ = dec1(in_batch(msg(PW.fld_varint(1, 16), PW.fld_bytes(12, snap))))
        assert bb["status"][0] == W.OK and mm["snapshot_host"][0] == host, snap


def _size_upper_limit_message(n_entries, cmd_len, snap_len):
    """Message.SizeUpperLimit (raft_optimized.go:1204-1216, Entry :70-76)."""
    return 16 * 12 + snap_len + n_entries * (16 + 16 * 7 + 16 + cmd_len)


def test_reference_size_upper_limits(wbuilt):
    """TestMessageSizeUpperLimit / TestMessageBatchSizeUpperLimit / TestEntrySizeUpperLimit
    (raftpb/raft_test.go:211-353): the marshalled size never exceeds SizeUpperLimit."""
    snap = (PW.fld_bytes(2, b"longfilepathisherexxxxxxxxxxxxxxxxx") + PW.fld_varint(3, MAX64) +
            PW.fld_varint(4, MAX64) + PW.fld_varint(5, MAX64) + PW.fld_bytes(6, PW.fld_varint(1, 0)))
    src = b"longaddressisherexxxxxxxxxxxxxxxxxxxxxxxxx"
    payload = np.frombuffer(src + snap + bytes(1024), np.uint8).copy()
    for n_msgs, n_ent, cmd in [(1, 1024, 1024), (4, 1024, 0), (1, 0, 0), (0, 0, 0)]:
        b = np.zeros(1, W.BATCH)
        b["deployment_id"] = MAX64
        b["bin_ver"] = 2**32 - 1
        b["source_off"], b["source_len"] = 0, len(src)
        b["n_msgs"] = n_msgs
        m = np.zeros(n_msgs, W.WMESSAGE)
        for f in ("to", "from", "cluster_id", "term", "log_term", "log_index", "commit", "hint", "hint_high"):
            m[f] = MAX64
        m["type"] = 4
        m["reject"] = 1
        m["snapshot_off"], m["snapshot_len"] = len(src), len(snap)
        m["n_entries"] = n_ent
        m["first_entry"] = 0
        e = np.zeros(n_ent, W.WENTRY)
        for f in ("term", "index", "key", "client_id", "series_id", "responded_to"):
            e[f] = MAX64
        e["type"] = 1
        e["cmd_off"], e["cmd_len"] = len(src) + len(snap), cmd
        out = PW.encode(payload, b, m, e)
        limit = 16 * 3 + len(src) + n_msgs * (16 + _size_upper_limit_message(n_ent, cmd, len(snap)))
        assert 0 < len(out) <= limit
        # and it decodes back (snapshot is non-zero: flagged for the host)
        bb = W.frames_table([0], [len(out)])
        bb, mm, ee = PW.decode(out, bb)
        assert bb["status"][0] == W.OK and len(mm) == n_msgs and len(ee) == n_msgs * n_ent
        assert (mm["snapshot_host"] == 1).all() and (mm["hint_high"] == MAX64).all()


def test_oracle_round_trip_random(wbuilt):
    payload, b, m, e = PW.make_records(30, 17, seed=5, snap_frac=0.1)
    out = PW.encode(payload, b, m, e)
    bb = W.frames_table(b["frame_off"], b["frame_len"])
    bb, mm, ee = PW.decode(out, bb)
    assert (bb["status"] == 0).all() and len(mm) == len(m) and len(ee) == len(e)
    for f in ("to", "from", "cluster_id", "term", "log_term", "log_index", "commit", "hint", "hint_high",
              "type", "reject", "n_entries"):
        assert (mm[f] == m[f]).all(), f
    for f in ("term", "index", "key", "client_id", "series_id", "responded_to", "type", "cmd_len"):
        assert (ee[f] == e[f]).all(), f
    for j in np.nonzero(e["cmd_len"])[0][:50]:
        a, n = int(ee["cmd_off"][j]), int(e["cmd_len"][j])
        assert out[a:a + n].tobytes() == payload[int(e["cmd_off"][j]):int(e["cmd_off"][j]) + n].tobytes()
    assert (mm["snapshot_host"] == (m["snapshot_len"] > 0)).all()
    assert (bb["deployment_id"] == b["deployment_id"]).all() and (bb["bin_ver"] == b["bin_ver"]).all()


def mutate(buf, rng, n):
    """Seeded corruptions of valid frames: byte flips, truncations, inserted bytes."""
    out = []
    for _ in range(n):
        x = bytearray(buf)
        k = rng.integers(0, 3)
        if k == 0 and x:
            for _ in range(rng.integers(1, 4)):
                x[rng.integers(0, len(x))] = rng.integers(0, 256)
        elif k == 1 and x:
            x = x[:rng.integers(0, len(x))]
        else:
            p = rng.integers(0, len(x) + 1)
            x[p:p] = bytes(rng.integers(0, 256, rng.integers(1, 4), dtype=np.uint8))
        out.append(bytes(x))
    return out


def fuzz_corpus(seed, n_frames):
    rng = np.random.default_rng(seed)
    payload, b, m, e = PW.make_records(n_frames, rng.integers(1, 6, n_frames), seed=seed, snap_frac=0.05)
    out = PW.encode(payload, b, m, e)
    frames = [out[int(o):int(o) + int(l)].tobytes() for o, l in zip(b["frame_off"], b["frame_len"])]
    corpus = []
    for f in frames:
        corpus.append(f)
        corpus += mutate(f, rng, 3)
    return PW.frames(*corpus)


def test_oracle_fuzz_is_total(wbuilt):
    """Every corrupted frame gets a status (no crash), and the error classes show up."""
    buf, b = fuzz_corpus(7, 200)
    bb, _, _ = PW.decode(buf, b)
    seen = set(int(s) for s in bb["status"])
    assert W.OK in seen and len(seen) >= 5, seen


# --------------------------------------------------------------- GPU parity --

def compare(buf, b_dev, m_dev, e_dev, b_ora, m_ora, e_ora):
    """Per frame: status and error fields always; values of OK frames and their records."""
    bad = []
    for f in W.BATCH_ERR_FIELDS:
        d = np.nonzero(b_dev[f] != b_ora[f])[0]
        if len(d):
            bad.append((f, int(d[0]), b_dev[f][d[0]], b_ora[f][d[0]]))
    ok = np.nonzero(b_ora["status"] == 0)[0]
    for f in W.BATCH_VALUE_FIELDS:
        if not (b_dev[f][ok] == b_ora[f][ok]).all():
            bad.append(("batch." + f,))
    if ok.size:
        jd = np.concatenate([np.arange(b_dev["first_msg"][i], b_dev["first_msg"][i] + b_dev["n_msgs"][i]) for i in ok])
        jo = np.concatenate([np.arange(b_ora["first_msg"][i], b_ora["first_msg"][i] + b_ora["n_msgs"][i]) for i in ok])
        jd, jo = jd.astype(np.int64), jo.astype(np.int64)
        for f in W.MSG_VALUE_FIELDS + ["snapshot_off", "snapshot_len"]:
            if not (m_dev[f][jd] == m_ora[f][jo]).all():
                bad.append(("msg." + f,))
        ne = m_ora["n_entries"][jo].astype(np.int64)
        if ne.sum():
            ed = np.concatenate([np.arange(a, a + n) for a, n in zip(m_dev["first_entry"][jd].astype(np.int64), ne)])
            eo = np.concatenate([np.arange(a, a + n) for a, n in zip(m_ora["first_entry"][jo].astype(np.int64), ne)])
            for f in W.ENTRY_FIELDS:
                if not (e_dev[f][ed] == e_ora[f][eo]).all():
                    bad.append(("entry." + f,))
    return bad


@pytest.mark.gpu
def test_gpu_decode_known_answers(wbuilt, gpu):
    codec = W.WireCodec(0)
    frames = [c[0] for c in ERROR_CASES.values()] + [in_batch(M0, M0)]
    buf, b = PW.frames(*frames)
    bd, md, ed = codec.unmarshal(buf, b.copy())
    bo, mo, eo = PW.decode(buf, b.copy())
    assert compare(buf, bd, md, ed, bo, mo, eo) == []
    for i, (name, c) in enumerate(ERROR_CASES.items()):
        assert int(bd["status"][i]) == c[1], name


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n_frames,mpb,steady", [(1, 64, 9, False), (2, 500, 40, True), (3, 3, 2000, True),
                                                      (4, 1, 1, False)])
def test_gpu_round_trip_parity(wbuilt, gpu, seed, n_frames, mpb, steady):
    """Device encode == oracle encode (bytes); device decode == oracle decode (records)."""
    codec = W.WireCodec(0)
    payload, b, m, e = PW.make_records(n_frames, mpb, seed=seed, steady=steady, snap_frac=0.02)
    bo = b.copy()
    out_o = PW.encode(payload, bo, m, e)
    bd = b.copy()
    out_d = codec.marshal(payload, bd, m, e)
    assert out_d.tobytes() == out_o.tobytes()
    assert (bd["frame_off"] == bo["frame_off"]).all() and (bd["frame_len"] == bo["frame_len"]).all()
    fr = W.frames_table(bo["frame_off"], bo["frame_len"])
    b1, m1, e1 = codec.unmarshal(out_o, fr.copy())
    b2, m2, e2 = PW.decode(out_o, fr.copy())
    assert compare(out_o, b1, m1, e1, b2, m2, e2) == []
    assert (b1["status"] == 0).all() and len(m1) == len(m) and len(e1) == len(e)


@pytest.mark.gpu
def test_gpu_fuzz_parity(wbuilt, gpu):
    """Corrupted frames: same status, error level, ordinal and field as the oracle;
    the frames that still decode carry the same records."""
    codec = W.WireCodec(0)
    for seed in (11, 12, 13):
        buf, b = fuzz_corpus(seed, 300)
        bd, md, ed = codec.unmarshal(buf, b.copy())
        bo, mo, eo = PW.decode(buf, b.copy())
        assert compare(buf, bd, md, ed, bo, mo, eo) == [], seed


@pytest.mark.gpu
def test_gpu_large_pass(wbuilt, gpu):
    """1M steady-state messages in 4k frames: device round trip, checked against the
    oracle on the whole pass."""
    codec = W.WireCodec(0)
    payload, b, m, e = PW.make_records(4096, 256, seed=21, steady=True)
    out = codec.marshal(payload, b, m, e)
    assert out.tobytes() == PW.encode(payload, b.copy(), m, e).tobytes()
    fr = W.frames_table(b["frame_off"], b["frame_len"])
    b1, m1, e1 = codec.unmarshal(out, fr.copy())
    b2, m2, e2 = PW.decode(out, fr.copy())
    assert compare(out, b1, m1, e1, b2, m2, e2) == []
    assert len(m1) == len(m) == 4096 * 256


@pytest.mark.gpu
@pytest.mark.parametrize("seg_shift", [None, "10", "16"])
def test_gpu_large_frame_segment_walk(wbuilt, gpu, seg_shift, monkeypatch):
    """Frames that average >= 64 KiB take the speculative segment walk (spec_segments +
    chain adoption in walk_frames): records, statuses and fields equal the oracle on
    steady and mixed large frames, and on seeded corruptions of them (flips,
    truncations and insertions anywhere in the frame shift or break the chains).
    GRW_SEG_SHIFT sweeps the segment size (1 KiB, the default 8 KiB, 64 KiB)."""
    if seg_shift:
        monkeypatch.setenv("GRW_SEG_SHIFT", seg_shift)
    codec = W.WireCodec(0)
    rng = np.random.default_rng(33)
    frames = []
    for seed, n_frames, mpb, steady in ((31, 5, 3000, True), (32, 4, 1500, False)):
        payload, b, m, e = PW.make_records(n_frames, mpb, seed=seed, steady=steady, snap_frac=0.02)
        out = PW.encode(payload, b, m, e)
        fr = W.frames_table(b["frame_off"], b["frame_len"])
        assert out.size // len(fr) >= 65536
        b1, m1, e1 = codec.unmarshal(out, fr.copy())
        b2, m2, e2 = PW.decode(out, fr.copy())
        assert compare(out, b1, m1, e1, b2, m2, e2) == [], seed
        assert (b1["status"] == 0).all() and len(m1) == len(m) and len(e1) == len(e)
        frames += [out[int(o):int(o) + int(l)].tobytes() for o, l in zip(b["frame_off"], b["frame_len"])]
    corpus = list(frames)
    for f in frames:
        corpus += mutate(f, rng, 3)
    buf, b = PW.frames(*corpus)
    assert buf.size // len(b) >= 65536
    bd, md, ed = codec.unmarshal(buf, b.copy())
    bo, mo, eo = PW.decode(buf, b.copy())
    assert compare(buf, bd, md, ed, bo, mo, eo) == []
    assert (bo["status"] != 0).any() and (bo["status"] == 0).any()


@pytest.mark.gpu
def test_gpu_encode_refuses_out_of_range_records(wbuilt, gpu):
    """grw_encode validates every record on the device before reading through it
    (ADVICE r01): an entry range past the entry array, a Cmd / Snapshot /
    SourceAddress past the payload buffer -> GR_EINVAL, nothing read out of range;
    the untouched records still encode after each refusal."""
    codec = W.WireCodec(0)
    payload, b, m, e = PW.make_records(8, 6, seed=5, steady=False, snap_frac=0.3)
    good = codec.marshal(payload, b.copy(), m, e)
    assert len(good) > 0
    P_ = len(payload)
    cases = []
    m1 = m.copy()
    m1["first_entry"][0] = len(e)  # entries past the array
    m1["n_entries"][0] = 1
    cases.append(("entries", b, m1, e))
    if len(e):
        e1 = e.copy()
        e1["cmd_off"][0], e1["cmd_len"][0] = P_ - 1, 2
        cases.append(("cmd", b, m, e1))
        e2 = e.copy()
        e2["cmd_off"][0], e2["cmd_len"][0] = 2**63, 1  # would wrap
        cases.append(("cmd wrap", b, m, e2))
    m2 = m.copy()
    m2["snapshot_off"][0], m2["snapshot_len"][0] = P_, 4
    cases.append(("snapshot", b, m2, e))
    b1 = b.copy()
    b1["source_off"][0], b1["source_len"][0] = P_ + 5, 1
    cases.append(("source", b1, m, e))
    for name, bb, mm, ee in cases:
        with pytest.raises(W.WireError, match=r"\(-1\)"):
            codec.marshal(payload, bb.copy(), mm, ee)
        assert codec.marshal(payload, b.copy(), m, e).tobytes() == good.tobytes(), name


@pytest.mark.gpu
def test_decode_refuses_overlapping_or_wrapping_frames(wbuilt, gpu):
    """grw_decode's host checks: a frame range that wraps 2^64 or two
    frames that overlap are refused before anything runs."""
    codec = W.WireCodec(0)
    payload, b, m, e = PW.make_records(4, 3, seed=6, steady=True)
    out = PW.encode(payload, b, m, e)
    fr = W.frames_table(b["frame_off"], b["frame_len"])
    bad = fr.copy()
    bad["frame_off"][1] = 2**64 - 4
    with pytest.raises(W.WireError, match=r"\(-1\)"):
        codec.unmarshal(out, bad)
    if len(fr) > 1:
        ov = fr.copy()
        ov["frame_off"][1] = ov["frame_off"][0] + 1
        ov["frame_len"][1] = 1
        with pytest.raises(W.WireError, match=r"\(-1\)"):
            codec.unmarshal(out, ov)
    b1, _, _ = codec.unmarshal(out, fr.copy())
    assert (b1["status"] == 0).all()
