"""Device-resident message exchange between passes (the transport's role).

In the reference every Replicate/ReplicateResp leaves a node through
``transport.Send`` (plugin/transport) and is delivered to the receiving
node's ``Peer.Handle`` on the next step. Here the engines of all GPUs write
their outgoing messages straight into mailbox "spaces" in HBM:

* ``local`` placement — all replicas of a group on one GPU: two spaces,
  ping-ponged; the kernel of pass k reads space k%2 and writes space (k+1)%2.
  No copy, no collective.
* ``spread`` placement — replica r of the groups homed on rank h lives on
  rank (h + r) % N, so replica r talks to replica j only across the rank
  offset (j - r) % N. The out space has one chunk per destination rank that
  some pair reaches (ordered by rank), the in space one per source rank, and
  one RCCL ``all_to_all_single`` with split sizes (0 for ranks no pair
  reaches) moves every mailbox across xGMI once per pass. At R = 3 that is
  4 of N chunks for N ≥ 5, and the spaces hold depth-3 mailboxes (the steady
  state's two Replicates per follower per pass plus a heartbeat on a tick; a
  fourth message escalates CAPACITY). The hot region (counts + compact
  Replicates + non-reject acks, 55 B per mailbox) crosses every pass; the cold
  region (132 B per mailbox) only when some mailbox holds another kind of
  message (gr_space_cold_used).

Peers on a rank are laid out replica-major: peer r*G + g is replica r of the
group (home = (rank - r) % N, index g), so a wave's accesses stay contiguous.
"""
import numpy as np

from . import populations as P

NOPOS = 0xFFFFFFFF


def pad_positions(positions):
    """gr_layout.h space_pad_positions: chunks hold a multiple of 64 mailboxes."""
    return (positions + 63) & ~63


def offset_pairs(R, N):
    """(sender replica r, receiver replica j) pairs per rank offset (j - r) % N."""
    pairs = {o: [] for o in range(N)}
    for r in range(R):
        for j in range(R):
            if j != r:
                pairs[(j - r) % N].append((r, j))
    return pairs


def spread_peer_ranks(R, N, rank):
    """(destination ranks, source ranks) of `rank`'s chunks, each sorted: the
    ranks some (r -> j) pair reaches at offset (j - r) % N, and back."""
    offs = [o for o, lst in offset_pairs(R, N).items() if lst]
    return sorted({(rank + o) % N for o in offs}), sorted({(rank - o) % N for o in offs})


def spread_routes(G, R, S, N, rank):
    """Route tables for spread placement on `rank`.

    Returns (in_pos [S][R*G], out_pos [S][R*G], positions per chunk). The
    sender on rank a writes its mailbox for (r -> j, group g) into the chunk
    of destination d = (a - r + j) % N (chunk index = d's place among a's
    destinations), position pair_index * G + g; all_to_all delivers it into
    the chunk of source a on rank d (a's place among d's sources), where the
    receiver (replica j, same group) reads the same position."""
    pairs = offset_pairs(R, N)
    per = max(len(v) for v in pairs.values())
    positions = per * G
    pc = pad_positions(positions)
    index = {}
    for o, lst in pairs.items():
        for k, rj in enumerate(lst):
            index[rj] = k
    dests, srcs = spread_peer_ranks(R, N, rank)
    dslot = {d: c for c, d in enumerate(dests)}
    sslot = {a: c for c, a in enumerate(srcs)}
    n = R * G
    g = np.arange(G, dtype=np.int64)
    in_pos = np.full((S, n), NOPOS, np.uint32)
    out_pos = np.full((S, n), NOPOS, np.uint32)
    for r in range(R):
        for j in range(R):
            if j == r:
                continue
            k = index[(r, j)]
            # sender: local replica r, slot j -> chunk d
            d = (rank - r + j) % N
            out_pos[j, r * G + g] = (dslot[d] * pc + k * G + g).astype(np.uint32)
            # receiver: local replica j, slot r <- chunk a (sender rank)
            a = (rank - j + r) % N
            in_pos[r, j * G + g] = (sslot[a] * pc + k * G + g).astype(np.uint32)
    return in_pos, out_pos, positions


def group_seed(seed, home):
    return [seed, home]


def spread_peers(G, R, N, rank, seed=2, **kw):
    """Peer records for `rank`: replica r of the G groups homed on (rank - r) % N.
    Every rank regenerates a home's groups from the same seed, so the replicas
    of one group agree wherever they are placed."""
    out = np.zeros(R * G, dtype=P.make_groups(1, R).dtype)
    for r in range(R):
        h = (rank - r) % N
        grp = P.make_groups(G, R, seed=int(np.random.SeedSequence(group_seed(seed, h)).generate_state(1)[0]), **kw)
        out[r * G:(r + 1) * G] = grp[r * G:(r + 1) * G]
    return out


class Exchange:
    """Spaces + routes for one rank; `step` launches one pass and exchanges."""

    def __init__(self, G, R, S, world, rank, placement, seed=2):
        self.G, self.R, self.S = G, R, S
        self.world, self.rank, self.placement = world, rank, placement
        self.n_peers = R * G
        self.leader_slots = np.arange(G)  # replica 0 of every hosted group leads
        if placement == "local":
            self.peers = P.make_groups(G, R, seed=int(np.random.SeedSequence(group_seed(seed, rank)).generate_state(1)[0]))
            self.in_pos, self.out_pos = P.Topology(G, R).loopback_routes(S)
            self.n_chunks = 1
            self.positions = self.n_peers * S
            self.depth = 4  # GR_C: nothing crosses a link, keep the full mailbox
            self.in_chunks = self.out_chunks = 1
        elif placement == "spread":
            self.peers = spread_peers(G, R, world, rank, seed=seed)
            self.in_pos, self.out_pos, self.positions = spread_routes(G, R, S, world, rank)
            self.dests, self.srcs = spread_peer_ranks(R, world, rank)
            self.n_chunks = len(self.dests)
            assert len(self.srcs) == self.n_chunks
            self.depth = 3  # two Replicates (or acks) + a heartbeat (or its ack) per pass
        else:
            raise ValueError(placement)

    def allocate(self, eng, device):
        import torch
        nbytes = eng.space_bytes(self.n_chunks, self.positions, self.depth)
        cb = eng.chunk_bytes(self.positions, self.depth)
        hb = eng.hot_chunk_bytes(self.positions, self.depth)
        assert nbytes == self.n_chunks * cb and 0 < hb < cb
        self.hot_region = self.n_chunks * hb  # hot chunks first, then the cold chunks
        self.cold_exchanges = 0
        if self.placement == "spread":  # all_to_all split sizes, bytes per peer rank
            self.hot_splits = ([hb if d in self.dests else 0 for d in range(self.world)],
                               [hb if a in self.srcs else 0 for a in range(self.world)])
            cold = cb - hb
            self.cold_splits = ([cold if d in self.dests else 0 for d in range(self.world)],
                                [cold if a in self.srcs else 0 for a in range(self.world)])
        a = torch.zeros(nbytes, dtype=torch.uint8, device=device)
        b = torch.zeros(nbytes, dtype=torch.uint8, device=device)
        return [a, b]

    def step(self, eng, spaces, k, stream, events=None):
        """One pass: kernel (optionally bracketed by `events`), then the exchange."""
        h = stream.cuda_stream
        if self.placement == "local":
            src, dst = spaces[k % 2], spaces[(k + 1) % 2]
        else:
            src, dst = spaces[0], spaces[1]
        if events is not None:
            events[0].record(stream)
        eng.step_device(src.data_ptr(), dst.data_ptr(), self.n_chunks, self.positions,
                        self.n_chunks, self.positions, self.n_peers, h, depth=self.depth)
        if events is not None:
            events[1].record(stream)
        if self.placement == "spread":
            # the hot region always; the cold region only when a mailbox needs it
            # (every steady-state message is hot-only: 37 B per depth-2 mailbox)
            hr = self.hot_region
            parts = [(slice(0, hr), self.hot_splits)]
            if eng.cold_used(spaces[1].data_ptr(), self.n_chunks, self.positions, self.depth, h):
                parts.append((slice(hr, None), self.cold_splits))
                self.cold_exchanges += 1
            for sl, (out_sp, in_sp) in parts:
                if self.world > 1:
                    import torch.distributed as dist
                    dist.all_to_all_single(spaces[0][sl], spaces[1][sl], output_split_sizes=in_sp,
                                           input_split_sizes=out_sp)
                else:
                    spaces[0][sl].copy_(spaces[1][sl])


def build_exchange(G, R, S, world, rank, placement, seed=2):
    return Exchange(G, R, S, world, rank, placement, seed=seed)
