"""Summarise a GR_WAVE_CLOCK dump (gr_engine.hip): the general kernel's waves of
the last pass an engine ran, each with its start and end clock (wall_clock64,
100 MHz on MI355X), lanes stepped, messages in, escalations and leader messages,
and the phase marks of its first round (loads done, run, store).

    GR_WAVE_CLOCK=gpurun_out/wc5.bin python tools/bench_configs.py --only 5 ...
    python tools/wave_clock.py gpurun_out/wc5.bin
"""
import sys

import numpy as np

WORDS = 8
TICK_NS = 10.0  # wall_clock64 at 100 MHz


def main(path):
    r = np.fromfile(path, dtype=np.uint64).reshape(-1, WORDS)
    r = r[:4096]  # the general kernel's region (the tick kernel's follows: tools/tick_clock.py)
    r = r[r[:, 1] > 0]
    if len(r) == 0:
        print("no waves recorded")
        return
    t0 = r[:, 0].astype(np.int64)
    t1 = r[:, 1].astype(np.int64)
    base = t0.min()
    start = (t0 - base) * TICK_NS / 1e3
    dur = (t1 - t0) * TICK_NS / 1e3
    end = (t1 - base) * TICK_NS / 1e3
    lanes, msgs, lmsg = (r[:, k].astype(np.int64) for k in (2, 3, 5))
    esc = (r[:, 4] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    cls = (r[:, 4] >> np.uint64(32)).astype(np.int64)  # the general list of the wave's first lane
    print(f"waves {len(r)}  lanes {lanes.sum()}  msgs {msgs.sum()}  escalated {esc.sum()}")
    print(f"kernel span {end.max():.1f} us; wave start p0/p50/p100 {start.min():.1f}/{np.median(start):.1f}/"
          f"{start.max():.1f} us")
    q = np.percentile(dur, [0, 10, 50, 90, 99, 100])
    print("wave duration us p0/p10/p50/p90/p99/p100: " + "/".join(f"{x:.1f}" for x in q))
    order = np.argsort(-dur)
    print("slowest waves: dur_us lanes msgs esc leader_msgs")
    for k in order[:12]:
        print(f"  {dur[k]:7.1f} {lanes[k]:4d} {msgs[k]:5d} {esc[k]:3d} {lmsg[k]:5d}")
    for name, v in (("lanes", lanes), ("msgs", msgs), ("leader_msgs", lmsg), ("escalated", esc)):
        if v.std() > 0:
            print(f"corr(duration, {name}) = {np.corrcoef(dur, v)[0, 1]:.2f}")
    # phase marks of each wave's first round (r[6]: loads done; r[7]: run << 32 | store)
    ph = r[:, 6] > 0
    if ph.any():
        pre = (r[ph, 6].astype(np.int64) - t0[ph]) * TICK_NS / 1e3
        run = (r[ph, 7] >> np.uint64(32)).astype(np.int64) * TICK_NS / 1e3
        sto = (r[ph, 7] & np.uint64(0xFFFFFFFF)).astype(np.int64) * TICK_NS / 1e3
        one = lanes[ph] <= 64
        rest = dur[ph] - pre - run - sto
        for name, v in (("setup + first loads", pre), ("run (messages, locals)", run), ("store", sto),
                        ("after store (single-round waves)", rest[one])):
            if len(v):
                print(f"phase {name:34s} p50 {np.median(v):7.1f}  p90 {np.percentile(v, 90):7.1f} us")
    # by handler class (gr_kernels.h general_bin: list = class x 2 + parity; class =
    # non-leader x 8 + higher-term x 4 + lower-term x 2 + full-record mailbox)
    print("by class of the wave's first lane: class waves p50_us p90_us msgs/lane")
    for c in sorted(set((cls // 2).tolist())):
        m = (cls // 2) == c
        names = ("leader" if c < 8 else "other") + (" higher" if c & 4 else "") + (" lower" if c & 2 else "") + \
            (" full" if c & 1 else "")
        print(f"  {c:2d} {names:28s} {m.sum():5d} {np.median(dur[m]):7.1f} {np.percentile(dur[m], 90):7.1f} "
              f"{msgs[m].sum() / max(lanes[m].sum(), 1):5.2f}")
    hist, edges = np.histogram(dur, bins=12)
    for h, a, b in zip(hist, edges[:-1], edges[1:]):
        print(f"  {a:7.1f}-{b:7.1f} us {h:5d} " + "#" * int(60 * h / max(hist.max(), 1)))


if __name__ == "__main__":
    main(sys.argv[1])
