"""Which mailboxes of a spread pass travel as full entries (not records) in the
compact exchange, and why: runs exchange.Pipeline (one rank, spread placement,
the exchange kept) with a Tick every third pass, copies each pass's out space
to the host, packs it with the host codec (gr_space_cx_pack_host, the device
kernel's logic) and prints, per pass, the record and full-entry counts and the
most common message signatures of the full entries.

    python tools/cx_census.py [--groups 4096] [--passes 9]
"""
import argparse
import collections
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=4096)
    ap.add_argument("--passes", type=int, default=9)
    ap.add_argument("--tick-every", type=int, default=3)
    a = ap.parse_args()
    import torch
    from dragonboat_amd import abi, populations as P
    from dragonboat_amd.engine import Engine, decode_space, cx_caps_array
    from dragonboat_amd import exchange as X
    R = 3
    pipe = X.Pipeline(a.groups, R, R, 1, 0, "spread", banks=1, exchange=True)

    def locals_fn(ex):
        return P.propose_locals(ex.n_peers, ex.leader_slots, pass_index=0)
    pipe.setup(Engine, torch.device("cuda", 0), 0, locals_fn)
    ex, eng = pipe.ex[0], pipe.engines[0]
    lib = eng.lib
    for k in range(a.passes):
        tk = 1 if a.tick_every and k % a.tick_every == a.tick_every - 1 else 0
        eng.set_locals(P.propose_locals(ex.n_peers, ex.leader_slots, pass_index=k, ticks=tk))
        # the pass alone (no exchange yet): the out space as the kernels wrote it
        s = pipe.streams[0]
        src, dst = pipe.spaces[0]
        ex.unpack(eng, pipe.spaces[0], s.cuda_stream) if k else None
        eng.step_device(src.data_ptr(), dst.data_ptr(), ex.n_chunks, ex.positions, ex.n_chunks, ex.positions,
                        ex.n_peers, s.cuda_stream, depth=ex.depth)
        torch.cuda.synchronize()
        out = dst.cpu().numpy()
        caps = np.array(ex.cx_send_caps, np.uint32)
        cb = int(lib.gr_space_cx_bytes(ex.n_chunks, ex.positions, ex.depth, caps.ctypes.data, ex.cx_scap))
        hcx = np.zeros(cb, np.uint8)
        assert lib.gr_space_cx_pack_host(out.ctypes.data, ex.n_chunks, ex.positions, ex.depth, hcx.ctypes.data,
                                         caps.ctypes.data, ex.cx_scap) == 0
        nrec, nside = X.cx_counts(hcx)
        # full entries: positions whose messages did not pack as records (host codec, position order)
        msgs = decode_space(out.copy(), ex.n_chunks, ex.positions, ex.depth, lost_ok=True)
        by = collections.defaultdict(list)
        for m in msgs:
            by[int(m["peer"])].append(m)
        # records: read the wave masks of the host-packed buffer
        L_waves = X.CX_HDR
        pc = X.pad_positions(ex.positions)
        nwv = pc // 64
        hdr = hcx[L_waves:L_waves + nwv * 24].reshape(nwv, 24)
        rec_mask = np.frombuffer(hdr[:, :8].tobytes(), np.uint64)
        sig = collections.Counter()
        for p, lst in by.items():
            if (int(rec_mask[p // 64]) >> (p % 64)) & 1:
                continue
            sig[tuple((int(m["type"]), int(m["n_entries"]), int(m["hint"] != 0), int(m["reject"])) for m in lst)] += 1
        print(f"pass {k} tick {tk}: records {nrec} full entries {nside} (capacity {ex.cx_scap})")
        for s_, n in sig.most_common(6):
            print("   ", n, s_)
        # the exchange proper (device codec): move and let the next pass unpack
        with torch.cuda.stream(s):
            ex.exchange(eng, pipe.spaces[0], s.cuda_stream)
        torch.cuda.synchronize()
    pipe.close()


if __name__ == "__main__":
    main()
