"""bench.py's N > 1 code path on one GPU: two ranks (processes) over gloo, each
running exchange.Pipeline (spread placement: replica r of a group homed on
rank h lives on rank (h + r) % 2, the mailboxes of other ranks cross through
all_to_all_single every pass, in the compact exchange's buffers or as the hot
region plus side buffers) on cuda:0. After every pass every rank's replicas
equal a single-process oracle run of the same groups (one population per bank
and home rank, messages routed inside each group), which each rank runs beside
its engines. RCCL refuses two ranks on one device, so the collective runs over
gloo (host copies); everything else is the RCCL path's code.

churn: BASELINE config 5's leader changes (p = 0.1 of the settled groups on
passes 1 and 4, applied to the oracle and to whichever rank holds each changed
replica) and a Tick on every replica every third pass, so step-downs, rejects,
multi-entry catch-ups, heartbeats and their acks -- full records -- cross ranks.
With the compact exchange every pass is compact, the tick passes' heartbeats
and acks as pattern records (round 6; round 5 exchanged them in the dense form)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, G, banks, passes, codec, churn, q, backend="gloo", collective=None, sizing="full",
            heavy_after=(0,), ticks=None):
    """One rank: Pipeline on cuda:0 beside the oracle, every pass. backend
    "nccl" with collective=True runs RCCL's async all_to_all_single even with
    one rank (tests/test_pipeline_rccl.py). sizing "full": room for a full entry
    at every position and full-depth mailboxes (churn); "default": the shipped
    capacities and depth, with `heavy` on the passes heavy_after says (offsets
    from each leader-change pass), CAPACITY escalations reported. ticks: a Tick
    on every replica every third pass (default: with churn)."""
    import torch
    import torch.distributed as dist
    from dragonboat_amd import abi, populations as P
    from dragonboat_amd.engine import Engine
    from dragonboat_amd.exchange import Pipeline, group_seed
    from oracle.pyoracle import OraclePopulation
    import parity
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    R = 3
    try:
        torch.cuda.set_device(0)
        dist.init_process_group(backend, rank=rank, world_size=world)
        # with churn and ticks few passes are steady: room for a full entry (compact
        # form) or a side entry (dense form) at every position, and full-depth
        # mailboxes (a new leader's catch-ups, proposal and heartbeats to one
        # follower in one pass overflow depth 3: CAPACITY, the host's to resolve)
        full = churn and sizing == "full"
        pipe = Pipeline(G, R, R, world, rank, "spread", banks=banks, seed=11, codec=codec,
                        cx_side=1.0 if full else None, depth=abi.GR_C if full else None, collective=collective)
        pipe.setup(Engine, torch.device("cuda", 0), 0)
        # the oracle: every bank's groups of every home, as one population each
        pops, msgs, topos = {}, {}, {}
        for b, ex in enumerate(pipe.ex):
            topos[b] = P.Topology(ex.G, R)
            for h in range(world):
                seed = int(np.random.SeedSequence(group_seed(11 + 7919 * b, h)).generate_state(1)[0])
                pops[(b, h)] = OraclePopulation(P.make_groups(ex.G, R, seed=seed), R)
                msgs[(b, h)] = np.zeros(0, abi.MESSAGE)
        rng = np.random.default_rng(100 + 0)  # the same draws on every rank
        bad, esc, first_esc = None, 0, None
        # heavy (dense) passes with the default sizing: the leader-change passes and
        # those heavy_after them; the tick passes travel compact (pattern records)
        changes = {1, 4} if churn else set()
        heavy_at = {k + d for k in changes for d in heavy_after} if sizing == "default" else set()
        capacity = 0
        ticks = churn if ticks is None else ticks
        for k in range(passes):
            tk = 1 if ticks and k % 3 == 2 else 0
            home_loc = {}
            for b, ex in enumerate(pipe.ex):
                Gb = ex.G
                for h in range(world):
                    pop = pops[(b, h)]
                    if churn and k in (1, 4):
                        cur = pop.export()
                        ch = P.inject_leader_change(cur, topos[b], 0.1, rng)
                        if len(ch):
                            pop.reload(ch, cur[ch])
                            mine = [(int(s) % Gb, int(s) // Gb) for s in ch if (h + int(s) // Gb) % world == rank]
                            if mine:
                                local = np.array([r * Gb + g for g, r in mine], np.uint32)
                                pipe.engines[b].load_peers(local, cur[[r * Gb + g for g, r in mine]])
                    st = pop.export()
                    leaders = np.nonzero(st["state"] == abi.LEADER)[0] if churn else np.arange(Gb)
                    home_loc[(b, h)] = P.propose_locals(R * Gb, leaders, pass_index=k if churn else 0, ticks=tk)
                # this rank's replica r of home (rank - r) % world takes that home's local input
                loc = np.zeros(R * Gb, abi.LOCAL)
                for r in range(R):
                    h = (rank - r) % world
                    sl = slice(r * Gb, (r + 1) * Gb)
                    loc[sl] = home_loc[(b, h)][sl]
                loc["peer"] = np.arange(R * Gb, dtype=np.uint32)
                pipe.engines[b].set_locals(loc)
            # "full" sizing: every pass compact, leader changes included (records and
            # full entries; the tick passes as pattern records). "default": heavy
            # where heavy_at says
            pipe.step(k, heavy=k in heavy_at)
            pipe.synchronize()
            print(f"rank {rank}/{world} pass {k}", flush=True)  # progress (pytest -s)
            for b, ex in enumerate(pipe.ex):
                Gb = ex.G
                dev = pipe.engines[b].sync(ex.n_peers)
                res = pipe.engines[b].collect_results(ex.n_peers)
                outs = {}
                for h in range(world):
                    # the oracle's mailboxes hold what the exchange's do (a fourth
                    # message escalates CAPACITY on both sides)
                    outs[h] = pops[(b, h)].step(msgs[(b, h)], home_loc[(b, h)], in_depth=ex.depth,
                                                out_depth=ex.depth)
                    msgs[(b, h)] = topos[b].route_messages(outs[h]["msgs"])
                for r in range(R):
                    h = (rank - r) % world
                    sl = slice(r * Gb, (r + 1) * Gb)
                    d = parity.compare_states(dev[sl], pops[(b, h)].export()[sl], R)
                    if d and bad is None:
                        bad = (k, b, r, d[:2])
                    # every escalation is the oracle's too (the churn's own: elections,
                    # full mailboxes); a mailbox the exchange lost would escalate
                    # CAPACITY at its reader where the oracle does not
                    de, oe = res["escalation"][sl], outs[h]["results"]["escalation"][sl]
                    capacity += int(((de == abi.ESC_NAMES.index("capacity")) & (oe != de)).sum())
                    mm = np.nonzero(de != oe)[0]
                    if len(mm) and esc == 0:
                        first_esc = (k, b, r, int(mm[0]), abi.ESC_NAMES[int(de[mm[0]])],
                                     abi.ESC_NAMES[int(oe[mm[0]])])
                    esc += len(mm)
        st = pipe.stats()
        pipe.close()
        dist.destroy_process_group()
        q.put((rank, bad, (esc, first_esc, capacity), st["leader_commits"], None))
    except Exception as e:  # reported to the test, never a hang
        import traceback
        q.put((rank, None, 0, 0, traceback.format_exc()))


@pytest.mark.parametrize("banks,codec,churn", [(1, "cx", False), (2, "cx", False), (2, "dense", False),
                                               (1, "cx", True), (2, "dense", True)])
def test_pipeline_world2_gloo_matches_oracle(gpu, banks, codec, churn):
    import torch.multiprocessing as mp
    world, G, passes = 2, 1000, 7 if churn else 6
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, G, banks, passes, codec, churn, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        for _ in procs:
            rank, bad, esc, commits, err = q.get(timeout=240)
            assert err is None, (rank, err)
            # esc: (count, first: pass, bank, replica, lane, device's, oracle's)
            assert bad is None, (rank, bad, esc)
            assert esc[0] == 0, (rank, esc)
            assert commits > 0
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()


def _run_world(world, G, banks, passes, codec, churn, **kw):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, G, banks, passes, codec, churn, q), kwargs=kw)
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = []
        for _ in procs:
            out.append(q.get(timeout=300))
        return out
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()


# Three to five ranks: every replica of a group on its own rank, as at N = 8
# (at world 2 replica 2 shares its home's rank); from N = 5 on a rank's chunks
# go to 4 of the N ranks (offsets 1, 2, N - 2, N - 1), as at N = 8, and the
# all-to-all's splits to the others are 0.
@pytest.mark.parametrize("world,G,churn", [(3, 4096, False), (3, 2048, True), (4, 2048, True),
                                           (4, 32768, True), (5, 4096, True)])
def test_pipeline_world_n_gloo_matches_oracle(gpu, world, G, churn):
    for rank, bad, esc, commits, err in _run_world(world, G, 1, 7 if churn else 5, "cx", churn):
        assert err is None, (rank, err)
        assert bad is None, (rank, bad, esc)
        assert esc[0] == 0, (rank, esc)
        assert commits > 0


# The shipped sizing (record capacities for the worst leader placement, full
# entries for 1/256 of the positions, depth 3) with a Tick on every replica every
# third pass and no heavy pass: heartbeats and acks cross 4 and 5 ranks as
# pattern records, and nothing escalates CAPACITY that the oracle does not.
@pytest.mark.parametrize("world", [4, 5])
def test_pipeline_world_n_default_sizing_ticks(gpu, world):
    for rank, bad, esc, commits, err in _run_world(world, 8192, 2, 7, "cx", False, sizing="default", ticks=True):
        assert err is None, (rank, err)
        assert bad is None, (rank, bad, esc)
        assert esc[0] == 0 and esc[2] == 0, (rank, esc)
        assert commits > 0
