"""The device-resident split schedule at BASELINE sizes, against the oracle
every pass (tests/devsim.DeviceLockstep: every peer, every mailbox, every
result, every escalation). This is the schedule bench.py and
tools/bench_configs.py time: gr_step_device over loopback spaces runs
gr_steady_kernel (closed-form steady lanes, quiet_step, tick routing), the role
instances over its wave lists (striding when the pass has more than 1,024
workgroups), the tick kernel and the general kernel; gr_step (test_gpu.py's
Lockstep) never launches the steady kernel."""
import numpy as np
import pytest

from dragonboat_amd import abi, populations as P
import devsim

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("Gl", [10_000, 10_048])
def test_device_config2_full_size(gpu, Gl):
    """BASELINE config 2: 10k x 3, one proposal per leader per pass (a small pass:
    the fused gr_small_kernel). Gl = 10,048: the layout tools/bench_configs.py times,
    replica blocks padded to whole waves with 48 idle groups (no input)."""
    G, R = 10_000, 3
    ls = devsim.DeviceLockstep(P.make_groups(Gl, R, seed=2), Gl, R)
    try:
        for k in range(8):
            ls.step(P.propose_locals(R * Gl, np.arange(G), pass_index=k))
        assert ls.stats["escalations"] == 0 and ls.stats["commits"] >= 5 * 3 * G
    finally:
        ls.close()


def test_device_config3_full_size(gpu):
    """BASELINE config 3: 100k x 5, 90% quiesced (QuiescedTick, closed form in the
    steady kernel), 10% active with a Tick per replica and a ReadIndex on the
    leader (steady-kernel tick routing, the tick kernel), HeartbeatResp dropped
    with p = 0.1, checkQuorum on half the groups."""
    G, R = 100_000, 5
    peers, active = P.config3(G, R)
    rng = np.random.default_rng(33)
    ls = devsim.DeviceLockstep(peers, G, R)
    try:
        for k in range(8):
            ls.step(P.config3_locals(G, R, active, k), drop_fn=lambda kk, m: P.drop_acks(m, 0.1, rng))
        assert ls.stats["ready"] > 0 and ls.stats["reencoded"] > 0
    finally:
        ls.close()


def test_device_config5_full_size(gpu):
    """BASELINE config 5: 100k x 3 (1,172 workgroups: the role instances stride),
    one proposal per current leader per pass, and from the second pass on a
    leader change with p = 0.1 per group (divergent suffixes, rejects,
    decreaseTo, truncation)."""
    G, R = 100_000, 3
    topo = P.Topology(G, R)
    rng = np.random.default_rng(5)
    ls = devsim.DeviceLockstep(P.make_groups(G, R, seed=5), G, R)
    try:
        for k in range(8):
            cur = ls.export()
            if k >= 1:
                ch = P.inject_leader_change(cur, topo, 0.1, rng)
                ls.inject(ch, cur[ch])
            ls.step(P.propose_locals(R * G, P.current_leaders(ls.export(), topo), pass_index=k))
        assert ls.stats["injected"] > 0 and ls.stats["commits"] > 0
    finally:
        ls.close()


@pytest.mark.parametrize("mode", ["1", "2"])
def test_tail_modes_churn(gpu, monkeypatch, mode):
    """The tail plan (gr_kernels.h TailPlan) forced each way on config-5 churn
    over the split schedule (20k x 3, leader changes p = 0.1 every pass):
    1 and 3 = the role instances every pass (round 4's schedule); 2 = never
    (the general kernel steps the listed waves and the retry lanes itself).
    Every peer, mailbox and result equals the oracle after every pass in each
    mode."""
    monkeypatch.setenv("GR_TAIL_MODE", mode)
    monkeypatch.setenv("GR_SPLIT_MIN_LANES", "1")
    monkeypatch.setenv("GR_SMALL_BLOCKS", "0")
    G, R = 20_000, 3
    topo = P.Topology(G, R)
    rng = np.random.default_rng(50 + int(mode))
    ls = devsim.DeviceLockstep(P.make_groups(G, R, seed=5), G, R)
    try:
        for k in range(8):
            cur = ls.export()
            if k >= 1:
                ch = P.inject_leader_change(cur, topo, 0.1, rng)
                ls.inject(ch, cur[ch])
            ls.step(P.propose_locals(R * G, P.current_leaders(ls.export(), topo), pass_index=k))
        assert ls.stats["injected"] > 0 and ls.stats["commits"] > 0
    finally:
        ls.close()


def test_device_config4_full_size_every_peer(gpu):
    """The headline population (1M x 3) on the device-resident path: every peer
    and every mailbox equal to the oracle after each of 3 passes."""
    G, R = 1_000_000, 3
    ls = devsim.DeviceLockstep(P.make_groups(G, R, seed=2), G, R)
    try:
        for k in range(3):
            ls.step(P.propose_locals(R * G, np.arange(G), pass_index=0))
        assert ls.stats["escalations"] == 0
    finally:
        ls.close()


def test_device_steady_leader_staggered_acks(gpu, monkeypatch):
    """Steady leaders (hinted by two steady passes of the split schedule) get
    acks at committed+1, +2 from one follower and +3 from the other: three
    commit broadcasts in one pass, more than the closed-form lane keeps, so it
    hands the lane to FastLane; state and mailboxes equal the
    oracle."""
    monkeypatch.setenv("GR_SPLIT_MIN_LANES", "1")
    monkeypatch.setenv("GR_SMALL_BLOCKS", "0")  # the split schedule, not the fused small-pass kernel
    G, R = 2048, 3
    ls = devsim.DeviceLockstep(P.make_groups(G, R, seed=21), G, R)
    try:
        for k in range(3):
            ls.step(P.propose_locals(R * G, np.arange(G), pass_index=k))
        cur = ls.export()
        c = cur["committed"][:G].copy()
        for r in range(R):
            cur["last_index"][r * G:(r + 1) * G] = c + np.uint64(3)
            cur["committed"][r * G:(r + 1) * G] = c
        L = cur[:G]
        L["remotes"]["next"][:, :R] = (c + np.uint64(4))[:, None]
        L["remotes"]["match"][:, 1:R] = c[:, None]
        L["remotes"]["match"][:, 0] = c + np.uint64(3)
        cur[:G] = L
        ls.inject(np.arange(R * G), cur)
        msgs = np.zeros(3 * G, abi.MESSAGE)
        for k, (slot, d) in enumerate(((1, 1), (1, 2), (2, 3))):
            m = msgs[k * G:(k + 1) * G]
            m["peer"] = np.arange(G, dtype=np.uint32)
            m["slot"] = slot
            m["type"] = abi.REPLICATE_RESP
            m["term"] = L["term"]
            m["log_index"] = c + np.uint64(d)
        ls.override_inbox(msgs[np.lexsort((np.arange(3 * G), msgs["slot"], msgs["peer"]))])
        ls.step(P.propose_locals(R * G, [], pass_index=9))
        assert np.all(ls.export()["committed"][:G] == c + np.uint64(3))
    finally:
        ls.close()


@pytest.mark.parametrize("G,split", [(10_000, False), (4096, True)])
def test_graph_replay_matches_oracle(gpu, monkeypatch, G, split):
    """Graph mode (gr_graph_capture / gr_graph_replay): two passes captured once,
    replayed three times through the C-ABI, then one pass by gr_step_device (the
    engine's parity is now odd: a replay is refused with GR_ESTATE and runs
    nothing), a second one, and one more replay: after every replay the state
    and the space the next pass reads equal the oracle's after the same number
    of passes. G = 10k is BASELINE config 2 (the fused small-pass
    kernel); the split schedule is forced on 4096 groups (steady kernel, role
    instances, general kernel in the graph)."""
    import torch
    from dragonboat_amd.engine import decode_space, GpuRaftError
    import parity
    if split:
        monkeypatch.setenv("GR_SPLIT_MIN_LANES", "1")
        monkeypatch.setenv("GR_SMALL_BLOCKS", "0")
    R = 3
    ls = devsim.DeviceLockstep(P.make_groups(G, R, seed=8), G, R)
    try:
        loc = P.propose_locals(R * G, np.arange(G), pass_index=0)
        ls.eng.set_locals(loc)
        a, b = ls.spaces
        g = ls.eng.graph_capture(a.data_ptr(), b.data_ptr(), 1, ls.positions, ls.n, n_passes=2, depth=ls.depth)
        pop = ls.pop
        msgs = np.zeros(0, abi.MESSAGE)
        stream = torch.cuda.current_stream().cuda_stream

        def replay_and_check(rep):
            nonlocal msgs
            ls.eng.graph_replay(g, stream)
            torch.cuda.synchronize()
            for _ in range(2):
                o = pop.step(msgs, loc)
                msgs = ls._route(o["msgs"])
            bad = parity.compare_states(ls.eng.sync(ls.n), pop.export(), R)
            assert not bad, (rep, bad[:3])
            got = decode_space(a.cpu().numpy(), 1, ls.positions, ls.depth)
            pos = got["peer"].astype(np.int64)
            got["peer"] = ls.inv[0][pos].astype(np.uint32)
            got["slot"] = ls.inv[1][pos].astype(np.uint8)
            bad = parity.compare_msgs(got, msgs)
            assert not bad, (rep, bad[:3])

        try:
            for rep in range(3):
                replay_and_check(rep)
            # a plain pass after the replays continues from their state (space a)
            ls.msgs = msgs
            ls.k = 0
            ls.step(loc)
            before = ls.eng.sync(ls.n)
            with pytest.raises(GpuRaftError):  # odd parity: refused, nothing ran
                ls.eng.graph_replay(g, stream)
            torch.cuda.synchronize()
            assert not parity.compare_states(ls.eng.sync(ls.n), before, R)
            ls.step(loc)  # even again: the live space is a
            msgs = ls.msgs
            replay_and_check(3)
        finally:
            ls.eng.graph_destroy(g)
        assert ls.stats["escalations"] == 0
    finally:
        ls.close()
