"""CPU baseline thread scaling on this host (run on the GPU box).

Times the oracle raft step (bench.py's cpu_baseline leg: the C++ restatement of
the reference Go step with its data structures) on config 4's shape at several
thread counts and prints one JSON line per count, plus the host's CPU limits
(nproc, affinity, cgroup cpu.max), so the baseline's T is chosen from data.

    python tools/cpu_scaling.py --threads 1,2,4,8,16,32 --seconds 3
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cgroup_cpu_max():
    for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(p) as f:
                return f.read().strip()
        except OSError:
            pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--groups", type=int, default=20000)
    ap.add_argument("--seconds", type=float, default=3.0)
    a = ap.parse_args()
    import numpy as np
    import bench
    from dragonboat_amd import populations as P
    info = bench.cpu_info()
    info["cgroup_cpu_max"] = cgroup_cpu_max()
    print(json.dumps({"host": info}), flush=True)
    R, G = 3, a.groups
    steady = lambda k, pop: P.propose_locals(R * G, np.arange(G), pass_index=k)
    for T in [int(x) for x in a.threads.split(",")]:
        peers = P.make_groups(G, R, seed=2)
        t0 = time.time()
        c, g, n = bench._oracle_rate(peers, P.Topology(G, R), R, steady, T, a.seconds)
        print(json.dumps({"threads": T, "commits_per_s": round(c), "groups_per_s": round(g), "passes": n,
                          "wall_s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
