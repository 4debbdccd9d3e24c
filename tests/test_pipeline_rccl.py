"""The exchange path BASELINE config 4 runs at N = 8, on one GPU: a one-rank
"nccl" (RCCL) process group, spread placement, and the exchange forced
through dist.all_to_all_single(..., async_op=True) on the bank's stream
(Exchange(collective=True)) instead of the one-rank device copy. So the code
that differs from every other test -- the RCCL collective issued async after
cx_pack / side_pack, work.wait() as a stream wait at the bank's next pass, then
cx_unpack / side_unpack and the pass on that stream -- runs under parity: after
every pass every replica equals the oracle (tests/test_pipeline_world2.py's
worker, world 1). Reference model: per-target batching of the messages that
exist (internal/transport/transport.go:399-476), groups sharded by
FixedPartitioner (internal/server/partition.go:38-40).

Cases: both codecs with config-5 churn and ticks (two banks, so one bank's
collective overlaps the other's pass), the shipped default sizing with ticks and
no heavy pass (capacity escalations reported and required to be zero), and BASELINE config 4's
1M x 3 population (two banks of 500k groups) in the compact form."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _run(G, banks, passes, codec, churn, sizing="full", heavy_after=(0,), timeout=240, ticks=None):
    import torch.multiprocessing as mp
    from test_pipeline_world2 import _worker
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    os.environ.setdefault("GR_VERIFY_HEAVY", "1")
    p = ctx.Process(target=_worker, args=(0, 1, port, G, banks, passes, codec, churn, q),
                    kwargs=dict(backend="nccl", collective=True, sizing=sizing, heavy_after=heavy_after,
                                ticks=ticks))
    p.start()
    try:
        rank, bad, esc, commits, err = q.get(timeout=timeout)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert err is None, err
    assert bad is None, (bad, esc)
    return esc, commits


@pytest.mark.parametrize("codec", ["cx", "dense"])
def test_rccl_exchange_churn_ticks(gpu, codec):
    esc, commits = _run(2000, 2, 8, codec, True)
    # esc: (mismatches, first: pass, bank, replica, lane, device's, oracle's; capacity)
    assert esc[0] == 0, esc
    assert commits > 0


def test_rccl_exchange_default_sizing_ticks(gpu):
    """The shipped capacities (records for the worst leader placement, full
    entries for 1/256 of the positions, depth 3) with a Tick on every replica
    every third pass and no pass declared heavy: the heartbeats and their acks
    travel as pattern records (round 6), so nothing is lost (a CAPACITY
    escalation the oracle does not have) and every replica stays equal to the
    oracle. (Round 5 exchanged tick passes in the dense form, whose side
    buffers hold the cold fields of 1/32 of the mailboxes, a third of them
    heartbeats on a tick pass.)"""
    esc, commits = _run(4096, 2, 9, "cx", False, sizing="default", ticks=True)
    assert esc[0] == 0 and esc[2] == 0, esc
    assert commits > 0


def test_rccl_exchange_config4_1m(gpu):
    """BASELINE config 4's population, 1M groups x 3 replicas, every replica
    compared with the oracle after each of 3 compact-exchange passes."""
    esc, commits = _run(1_000_000, 2, 3, "cx", False, timeout=420)
    assert esc[0] == 0, esc
    assert commits > 0
