"""Device wire-codec throughput: MessageBatch.Unmarshal and
MarshalTo of one transport pass of steady-state raft messages, inputs resident
in HBM, beside the oracle's CPU decode of the same frames.

  python tools/bench_wire.py [--frames 16384] [--per-frame 256] [--reps 20]

Prints one JSON line. Roofline: bytes moved per pass (frames read + records
written for decode; records read + frames written for encode) over the device
time of the pass (HIP events inside libgrwire.so), against the 8 TB/s spec.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16384)
    ap.add_argument("--per-frame", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-baseline", default="on")
    args = ap.parse_args()

    import torch
    from dragonboat_amd import wire as W
    from oracle import pywire as PW

    torch.cuda.set_device(0)
    payload, b, m, e = PW.make_records(args.frames, args.per_frame, seed=42, steady=True)
    frames = PW.encode(payload, b, m, e)  # the oracle writes the input frames
    n, nm, ne = len(b), len(m), len(e)
    codec = W.WireCodec(0)
    dev = torch.device("cuda:0")
    d_buf = torch.from_numpy(frames).to(dev)
    fr = W.frames_table(b["frame_off"], b["frame_len"])
    d_fr = torch.from_numpy(fr.view(np.uint8)).to(dev)
    d_msgs = torch.empty(nm * W.WMESSAGE.itemsize, dtype=torch.uint8, device=dev)
    d_ents = torch.empty(max(ne, 1) * W.WENTRY.itemsize, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def decode():
        return codec.unmarshal_device(d_buf.data_ptr(), frames.size, d_fr.data_ptr(), n, d_msgs.data_ptr(), nm,
                                      d_ents.data_ptr(), ne)

    for _ in range(3):
        decode()
    dt, wall = [], []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        got = decode()
        wall.append(time.perf_counter() - t0)
        dt.append(codec.timing())
    assert got == (nm, ne), got
    # parity screen on the device output of the timed passes
    md = d_msgs.cpu().numpy().view(W.WMESSAGE)
    fo = fr.copy()
    bo, mo, eo = PW.decode(frames, fo)
    bd = d_fr.cpu().numpy().view(W.BATCH)
    for f in ("term", "log_index", "commit", "type", "n_entries", "msg_off"):
        assert (md[f] == mo[f]).all(), f
    assert (bd["status"] == 0).all()
    dec_ms = float(np.median([t["total_ms"] for t in dt]))
    dec_bytes = frames.size + nm * W.WMESSAGE.itemsize + ne * W.WENTRY.itemsize + n * W.BATCH.itemsize

    # encode: records resident in HBM -> frames
    d_payload = torch.from_numpy(payload).to(dev)
    d_b = torch.from_numpy(b.view(np.uint8).copy()).to(dev)
    d_m = torch.from_numpy(m.view(np.uint8)).to(dev)
    d_e = torch.from_numpy(e.view(np.uint8)).to(dev)
    d_out = torch.empty(frames.size + 16, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def encode():
        return codec.marshal_device(d_payload.data_ptr(), payload.size, d_b.data_ptr(), n, d_m.data_ptr(), nm,
                                    d_e.data_ptr(), ne, d_out.data_ptr(), d_out.numel())

    for _ in range(3):
        encode()
    et = []
    for _ in range(args.reps):
        encode()
        et.append(codec.timing())
    out = d_out[:frames.size].cpu().numpy()
    assert out.tobytes() == frames.tobytes(), "device encode != oracle encode"
    enc_ms = float(np.median([t["total_ms"] for t in et]))
    enc_bytes = frames.size + nm * W.WMESSAGE.itemsize + ne * W.WENTRY.itemsize + n * W.BATCH.itemsize + \
        ne * 16

    rec = {
        "metric": "raft wire codec: messages decoded/s (MessageBatch.Unmarshal, HBM-resident frames)",
        "value": nm / (dec_ms * 1e-3), "unit": "messages/s", "higher_is_better": True, "dtype": "u8",
        "config": {"workload": f"{n} frames x {args.per_frame} steady-state messages "
                               f"(Replicate/ReplicateResp/Heartbeat/HeartbeatResp, 16-B Cmd)",
                   "frames": n, "messages": nm, "entries": ne, "frame_bytes": int(frames.size)},
        "decode": {"ms": dec_ms, "phases_ms": {k: float(np.median([t[k] for t in dt]))
                                               for k in ("walk_ms", "scan_ms", "message_ms", "entry_ms")},
                   "wall_ms_incl_host_sync": float(np.median(wall)) * 1e3,
                   "bytes": dec_bytes, "GBs": dec_bytes / dec_ms / 1e6},
        "encode": {"ms": enc_ms, "messages_per_s": nm / (enc_ms * 1e-3), "bytes": enc_bytes,
                   "GBs": enc_bytes / enc_ms / 1e6,
                   "phases_ms": {"size": float(np.median([t["walk_ms"] for t in et])),
                                 "write": float(np.median([t["entry_ms"] for t in et]))}},
        "roofline": {"bound": "hbm", "achieved": dec_bytes / dec_ms / 1e6, "peak": 8000.0, "unit": "GB/s",
                     "frac": dec_bytes / dec_ms / 1e6 / 8000.0, "traffic": None, "kernel": "decode pass"},
    }
    if args.cpu_baseline == "on":
        rate, reps = PW.decode_bench(frames, fr, args.cpu_threads, args.cpu_seconds)
        rate1, reps1 = PW.decode_bench(frames, fr, 1, max(2.0, args.cpu_seconds / 4))
        rec["cpu_baseline"] = {"value": rate, "unit": "messages/s", "cores": args.cpu_threads, "kind": "port",
                               "sample": f"the same {n} frames, {reps} passes, oracle MessageBatch.Unmarshal "
                                         f"restatement, frames split over threads",
                               "single_thread": rate1}
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
