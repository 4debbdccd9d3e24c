"""Parity workloads run by tests/test_sanitizers.py in a child process under
ASAN + UBSAN (the sanitized oracle or host lane selected with GR_ORACLE_LIB /
GR_HOSTLANE_LIB, the matching runtime preloaded). Exits non-zero on divergence;
the sanitizers abort the process on the first error."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]

from dragonboat_amd import abi, populations as P  # noqa: E402
import simulate as SIM  # noqa: E402


def main():
    G, R = 120, 3
    topo = P.Topology(G, R)
    rng = np.random.default_rng(7)
    # leader churn with truncations (config 5's generator)
    SIM.simulate(SIM.HostlaneBackend, P.make_groups(G, R, seed=7), topo, 10,
                 lambda k, st: P.propose_locals(R * G, P.current_leaders(st, topo), pass_index=k),
                 inject_fn=lambda k, cur: P.inject_leader_change(cur, topo, 0.15, rng))

    # ticks, ReadIndex, heartbeats, CheckQuorum
    def lf(k):
        loc = P.propose_locals(R * G, np.arange(G), pass_index=k)
        loc["ticks"] = rng.integers(0, 3, R * G)
        loc["read_index"] = rng.random(R * G) < 0.3
        loc["read_ctx_low"] = rng.integers(1, 2**63, R * G, dtype=np.uint64)
        loc["read_ctx_high"] = k
        return loc
    SIM.simulate(SIM.HostlaneBackend, P.make_groups(G, R, seed=8, check_quorum=True), topo, 10, lf)
    # BASELINE config 3's shape (R = 5, quiesced majority, dropped acks)
    G3 = 200
    peers, active = P.config3(G3, 5)
    rng3 = np.random.default_rng(33)
    SIM.simulate(SIM.HostlaneBackend, peers, P.Topology(G3, 5), 6, lambda k: P.config3_locals(G3, 5, active, k),
                 slots=5, drop_fn=lambda k, m: P.drop_acks(m, 0.1, rng3))
    maps = open("/proc/self/maps").read()
    for var in ("GR_ORACLE_LIB", "GR_HOSTLANE_LIB"):
        if os.environ.get(var):
            assert os.path.basename(os.environ[var]) in maps, f"{var} not loaded"
    print("san workload ok")


if __name__ == "__main__":
    main()
