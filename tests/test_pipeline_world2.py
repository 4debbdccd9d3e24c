"""bench.py's N > 1 code path on one GPU: two ranks (processes) over gloo, each
running exchange.Pipeline (spread placement: replica r of a group homed on
rank h lives on rank (h + r) % 2, the mailboxes of other ranks cross through
all_to_all_single every pass, cold fields through the side buffers) on cuda:0.
After every pass every rank's replicas equal a single-process oracle run of
the same groups (one population per bank and home rank, messages routed
inside each group). RCCL refuses two ranks on one device, so the collective
runs over gloo (host copies); everything else is the RCCL path's code."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, G, banks, passes, q):
    import torch
    import torch.distributed as dist
    from dragonboat_amd.engine import Engine
    from dragonboat_amd.exchange import Pipeline
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pipe = Pipeline(G, 3, 3, world, rank, "spread", banks=banks, seed=11)
        pipe.setup(Engine, torch.device("cuda", 0), 0)
        states = []
        for k in range(passes):
            pipe.step(k)
            pipe.synchronize()
            states.append([eng.sync(ex.n_peers) for ex, eng in zip(pipe.ex, pipe.engines)])
        st = pipe.stats()
        pipe.close()
        dist.destroy_process_group()
        q.put((rank, states, st["escalations"], None))
    except Exception as e:  # reported to the test, never a hang
        q.put((rank, None, 0, repr(e)))


@pytest.mark.parametrize("banks", [1, 2])
def test_pipeline_world2_gloo_matches_oracle(gpu, banks):
    import torch.multiprocessing as mp
    from dragonboat_amd import abi, populations as P
    from dragonboat_amd.exchange import Exchange, group_seed
    from oracle.pyoracle import OraclePopulation
    import parity
    world, G, passes, R = 2, 1000, 6, 3
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, G, banks, passes, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            rank, states, esc, err = q.get(timeout=240)
            assert err is None, (rank, err)
            assert esc == 0
            res[rank] = states
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    # bank layout as Pipeline builds it (sizes and seeds per bank)
    from dragonboat_amd.exchange import Pipeline
    layout = Pipeline(G, R, R, world, 0, "spread", banks=banks, seed=11)
    topo = {}
    for b, ex in enumerate(layout.ex):
        seed = 11 + 7919 * b
        Gb = ex.G
        tp = P.Topology(Gb, R)
        for h in range(world):
            peers = P.make_groups(Gb, R, seed=int(np.random.SeedSequence(group_seed(seed, h)).generate_state(1)[0]))
            pop = OraclePopulation(peers, R)
            msgs = np.zeros(0, abi.MESSAGE)
            seq = []
            for k in range(passes):
                o = pop.step(msgs, P.propose_locals(R * Gb, np.arange(Gb), pass_index=0))
                seq.append(pop.export())
                msgs = tp.route_messages(o["msgs"])
            topo[(b, h)] = seq
    for rank in range(world):
        for k in range(passes):
            for b, ex in enumerate(layout.ex):
                dev = res[rank][k][b]
                Gb = ex.G
                for r in range(R):
                    h = (rank - r) % world
                    sl = slice(r * Gb, (r + 1) * Gb)
                    bad = parity.compare_states(dev[sl], topo[(b, h)][k][sl], R)
                    assert not bad, (rank, k, b, r, bad[:2])
    assert all(int(res[r][-1][0]["committed"][:10].min()) > int(res[r][0][0]["committed"][:10].min()) for r in res)
