"""GPU parity: the HIP kernel (libgpuraft.so through the C-ABI) against the
oracle, bit-exact, on the host-staged path (gr_step) and the device-resident
path (gr_step_device + mailbox spaces)."""
import os

import numpy as np
import pytest

from dragonboat_amd import populations as P
import simulate as SIM

pytestmark = pytest.mark.gpu


def _loaded_native():
    with open("/proc/self/maps") as f:
        return "libgpuraft.so" in f.read()


def test_smoke(gpu):
    import __graft_entry__ as ge
    ge.smoke()
    assert _loaded_native()


def _sim(G, passes, seed, locals_fn=None, inject_p=0.0, **mk):
    R = 3
    peers = P.make_groups(G, R, seed=seed, **mk)
    topo = P.Topology(G, R)
    rng = np.random.default_rng(seed)
    lf = locals_fn or (lambda k: P.propose_locals(R * G, np.arange(G), pass_index=k))
    inj = (lambda k, cur: P.inject_leader_change(cur, topo, inject_p, rng)) if inject_p else None
    return SIM.simulate(SIM.GpuBackend, peers, topo, passes, lf, inject_fn=inj)


def test_gpu_steady_state(gpu):
    st = _sim(1000, 6, seed=3)
    assert st["escalations"] == 0 and st["commits"] > 0


def test_gpu_leader_change_churn(gpu):
    st = _sim(500, 16, seed=5, inject_p=0.1)
    assert st["commits"] > 0


@pytest.mark.parametrize("check_quorum", [False, True])
def test_gpu_ticks_and_read_index(gpu, check_quorum):
    G, R = 256, 3
    rng = np.random.default_rng(9)

    def lf(k):
        loc = P.propose_locals(R * G, np.arange(G), pass_index=k)
        loc["ticks"] = rng.integers(0, 3, R * G)
        loc["read_index"] = rng.random(R * G) < 0.3
        loc["read_ctx_low"] = rng.integers(1, 2**63, R * G, dtype=np.uint64)
        loc["read_ctx_high"] = k
        loc["propose_entries"] = np.where(rng.random(R * G) < 0.5, loc["propose_entries"], 0)
        return loc
    _sim(G, 10, seed=7, locals_fn=lf, check_quorum=check_quorum)


@pytest.mark.parametrize("placement", ["local", "spread"])
def test_device_resident_path(gpu, placement):
    """The bench path: spaces in HBM, routes bound once, locals bound once."""
    import devsim
    final = devsim.run_device(777, 3, 6, placement=placement)
    assert np.all(final["committed"][:777] > 2**32)


def test_bench_runs(gpu):
    """bench.py's contract on a small population (JSON line with roofline)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--groups", "20000", "--steps", "5",
                        "--warmup", "3", "--cpu-baseline", "off"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["value"] > 0 and line["escalations"] == 0
    assert line["roofline"]["achieved"] > 0


def test_gpu_config3_read_index_quiesced(gpu):
    """BASELINE config 3 shape on the GPU (R=5, slots=5 kernels)."""
    R, G = 5, 1000
    peers, active = P.config3(G, R)
    topo = P.Topology(G, R)
    rng = np.random.default_rng(33)
    st = SIM.simulate(SIM.GpuBackend, peers, topo, 8, lambda k: P.config3_locals(G, R, active, k),
                      slots=R, drop_fn=lambda k, m: P.drop_acks(m, 0.1, rng))
    assert st["ready"] > 0
