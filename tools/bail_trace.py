"""Why lanes leave the lean kernels: a CPU diagnostic over the host build of the
lane code (tests/native/hostlane.hip built with -DGR_BAIL_TRACE).

Runs a BASELINE config population through the Lockstep (host lane vs oracle, every
pass checked) with the hints the device would give, and prints
  - per gr_fast.h source line, how many lanes that GF_BAIL condition handed over
    (the first failing condition of each lane);
  - the general/tick lane's branch hits (gr_cover.h) over the same passes.

    python tools/bail_trace.py --config 5 --groups 20000 --passes 8
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
TRACE_LIB = os.path.join(ROOT, "tests", "_build", "libhostlane_trace.so")


def build():
    from dragonboat_amd import build as B
    src = os.path.join(ROOT, "tests", "native", "hostlane.hip")
    if B._stale(TRACE_LIB, B.ENGINE_DEPS + [src]):
        subprocess.check_call([B.HIPCC, "--cuda-host-only", "-O2", "-g", "-std=c++17", "-fPIC", "-shared",
                               "-DGR_COVERAGE", "-DGR_BAIL_TRACE", "-I" + os.path.join(ROOT, "include"),
                               "-I" + os.path.join(ROOT, "dragonboat_amd", "csrc"), src, "-o", TRACE_LIB])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="5")
    ap.add_argument("--groups", type=int, default=20000)
    ap.add_argument("--passes", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3, help="passes before injection starts / counting")
    a = ap.parse_args()
    build()
    os.environ["GR_HOSTLANE_LIB"] = TRACE_LIB
    import numpy as np
    from dragonboat_amd import populations as P
    import simulate as SIM
    from oracle import pyoracle
    lib = pyoracle.hostlane_lib()
    lib.hl_coverage_names.restype = ctypes.c_char_p
    lib.hl_bail_trace.restype = ctypes.c_uint32
    lib.hl_true_hints(1)
    G = a.groups
    if a.config == "5":
        R = 3
        peers = P.make_groups(G, R, seed=5)
        topo = P.Topology(G, R)
        rng = np.random.default_rng(5)
        inj = lambda k, cur: P.inject_leader_change(cur, topo, 0.1, rng) if k >= a.warmup else None
        lf = lambda k, st: P.propose_locals(R * G, P.current_leaders(st, topo), pass_index=k)
        drop = None
    elif a.config == "3":
        R = 5
        peers, act = P.config3(G, R)
        topo = P.Topology(G, R)
        rng = np.random.default_rng(3)
        inj = None
        lf = lambda k: P.config3_locals(G, R, act, k)
        drop = lambda k, m: P.drop_acks(m, 0.1, rng)
    else:
        R = 3
        peers = P.make_groups(G, R, seed=2)
        topo = P.Topology(G, R)
        inj = None
        lf = lambda k: P.propose_locals(R * G, np.arange(G), pass_index=k)
        drop = None
    names = lib.hl_coverage_names().decode().strip(",").split(",")
    cov0 = np.zeros(len(names), np.uint64)
    lines = np.zeros(256, np.int32)
    counts = np.zeros(256, np.uint64)

    def snap():
        c = np.zeros(len(names), np.uint64)
        lib.hl_coverage(c.ctypes.data_as(ctypes.c_void_p), len(names))
        return c

    state = {"k": 0}

    def lf2(k, st=None):
        if k == a.warmup:  # start counting
            lib.hl_bail_trace(lines.ctypes.data_as(ctypes.c_void_p), counts.ctypes.data_as(ctypes.c_void_p), 256)
            cov0[:] = snap()
            f, b = ctypes.c_uint64(), ctypes.c_uint64()
            lib.hl_counters(ctypes.byref(f), ctypes.byref(b))
            state["fb0"] = (f.value, b.value)
        return lf(k, st) if lf.__code__.co_argcount == 2 else lf(k)
    st = SIM.simulate(SIM.HostlaneBackend, peers, topo, a.passes, lf2, slots=R, inject_fn=inj, drop_fn=drop)
    n = lib.hl_bail_trace(lines.ctypes.data_as(ctypes.c_void_p), counts.ctypes.data_as(ctypes.c_void_p), 256)
    f, b = ctypes.c_uint64(), ctypes.c_uint64()
    lib.hl_counters(ctypes.byref(f), ctypes.byref(b))
    f0, b0 = state["fb0"]
    npass = a.passes - a.warmup
    print(f"config {a.config}: {G} groups x {R}, {npass} counted passes; lanes per pass: lean "
          f"{(f.value - f0) / npass:.0f}, handed over {(b.value - b0) / npass:.0f}; escalations {st['escalations']} "
          f"{st['esc_reasons']}")
    src = open(os.path.join(ROOT, "dragonboat_amd", "csrc", "gr_fast.h")).read().split("\n")
    print("first GF_BAIL per handed-over lane (gr_fast.h line: lanes/pass):")
    for k in np.argsort(-counts[:n].astype(np.int64)):
        if lines[k] >= 100000:  # (type, flags) of a non-uniform mailbox a leader bailed on
            print(f"  nonu type {(lines[k] - 100000) // 1000} flags {lines[k] % 1000:#x}: {counts[k] / npass:9.0f}")
            continue
        print(f"  {lines[k]:4d}: {counts[k] / npass:9.0f}  {src[lines[k] - 1].strip()[:110]}")
    cov = snap() - cov0
    print("general / tick lane branch hits per pass:")
    for k in np.argsort(-cov.astype(np.int64)):
        if cov[k]:
            print(f"  {names[k]:28s} {cov[k] / npass:9.0f}")


if __name__ == "__main__":
    main()
