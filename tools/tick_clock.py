"""Phases of the tick kernel's waves from a GR_WAVE_CLOCK dump (second region,
gr_kernels.h gr_tick_kernel): per wave its start, end, lanes, leader entries and
the marks of its first entries (round-1 loads in, round-2 loads in, stores
issued). wall_clock64 runs at 100 MHz (10 ns per tick).

    GR_WAVE_CLOCK=gpurun_out/wclk.bin python tools/bench_configs.py --only 3
    python tools/tick_clock.py gpurun_out/wclk.bin
"""
import sys

import numpy as np

SLOTS, WORDS, TICK_NS = 4096, 8, 10.0


def main():
    a = np.fromfile(sys.argv[1], np.uint64).reshape(2, SLOTS, WORDS)[1]
    a = a[a[:, 0] != 0]
    if not len(a):
        raise SystemExit("no tick-kernel waves recorded")
    t0, t1, nl, nld, r1, r2, st = (a[:, k].astype(np.int64) for k in range(7))
    base = t0.min()
    print(f"waves {len(a)}, lanes {nl.sum()}, span {(t1.max() - base) * TICK_NS / 1e3:.2f} us")
    for name, m in (("follower", nld == 0), ("leader", nld > 0)):
        if not m.any():
            continue
        ph = np.stack([r1 - t0, r2 - r1, st - r2, t1 - st, t0 - base, t1 - base], 1)[m] * TICK_NS / 1e3
        q = np.percentile(ph, [50, 90, 100], axis=0)
        print(f"{name:8s} waves {m.sum():5d}   (us)   round1  round2  compute+stores  tail   start   end")
        for lab, row in zip(("p50", "p90", "max"), q):
            print(f"   {lab:5s}" + "".join(f"{v:8.2f}" for v in row))


if __name__ == "__main__":
    main()
