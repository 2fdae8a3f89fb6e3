"""Multi-rank sharding logic on CPU (gloo, world_size 2; the pipelined
assembly also at 4 and 8 ranks).

The per-rank compute here is the CPU oracle (test infrastructure standing in
for the rank's GPU kernel); what is under test is the product's sharding
plan and its collectives: the output all-gather must reproduce the
single-device FedAvg bit for bit, and the Krum partial all-reduce must give
the same distance matrix and selection as the unsharded computation.
"""
import os
import socket
from collections import OrderedDict

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n=7, keys=((5, 3), (1, ), (130, ), (33, 2))):
    rng = np.random.default_rng(11)
    clients = []
    for i in range(n):
        d = OrderedDict(('k%d' % j, rng.standard_normal(s).astype(np.float32))
                        for j, s in enumerate(keys))
        clients.append((int(rng.integers(1, 100)), d))
    return clients


def _flat(d):
    return np.concatenate([v.ravel() for v in d.values()])


def _worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from federatedscope_amd.core.sharding import (allreduce_segsq,
                                                      assemble,
                                                      local_segments,
                                                      shard_ranges)
        clients = _data()
        n = len(clients)
        X = np.stack([_flat(d) for _, d in clients])
        P = X.shape[1]
        ranges = shard_ranges(P, world, align=16)
        lo, hi = ranges[rank]
        # FedAvg on this rank's range (oracle = the rank's kernel)
        w = O.fedavg_weights([s for s, _ in clients])
        shard = O.para_weighted_avg([(s, {'w': X[i, lo:hi]})
                                     for i, (s, _) in enumerate(clients)],
                                    weights=w)['w']
        full = assemble(torch.from_numpy(shard.copy()), ranges, P).numpy()
        want = O.para_weighted_avg([(s, {'w': X[i]}) for i, (s, _) in
                                    enumerate(clients)], weights=w)['w']
        fedavg_ok = full.tobytes() == want.tobytes()
        # Krum partials: per-key squared distances over this rank's range
        sizes = [v.size for v in clients[0][1].values()]
        offs = np.concatenate([[0], np.cumsum(sizes)]).tolist()
        loc = local_segments(offs, lo, hi)
        Xl = X[:, lo:hi].astype(np.float64)
        segsq = np.zeros((len(sizes), n, n))
        for s in range(len(sizes)):
            blk = Xl[:, loc[s]:loc[s + 1]]
            for a in range(n):
                segsq[s, a] = ((blk - blk[a]) ** 2).sum(1)
        t = torch.from_numpy(segsq)
        allreduce_segsq(t)
        D = np.sqrt(t.numpy()).astype(np.float32).sum(0, dtype=np.float32)
        np.fill_diagonal(D, np.inf)
        Dref = O.krum_distance_matrix([d for _, d in clients])
        off = ~np.eye(n, dtype=bool)
        krum_ok = bool(np.allclose(D[off], Dref[off], rtol=1e-5)) and \
            O.krum_select(O.krum_scores(D, 1), 3) == \
            O.krum_select(O.krum_scores(Dref, 1), 3)
        q.put((rank, fedavg_ok, krum_ok, (lo, hi)))
    finally:
        dist.destroy_process_group()


def test_sharded_fedavg_and_krum_world2():
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert all(r[1] for r in res), res   # bit-exact assembled FedAvg
    assert all(r[2] for r in res), res   # Krum matrix + selection
    assert res[0][3][1] == res[1][3][0]  # contiguous ranges


def test_shard_ranges_and_local_segments():
    from federatedscope_amd.core.sharding import local_segments, shard_ranges
    r = shard_ranges(1000, 3, align=64)
    assert r == [(0, 384), (384, 768), (768, 1000)]
    assert all(lo % 64 == 0 for lo, _ in r)
    assert shard_ranges(10, 4, align=64) == [(0, 10), (10, 10), (10, 10),
                                            (10, 10)]
    offs = [0, 100, 400, 1000]
    assert local_segments(offs, 384, 768) == [0, 0, 16, 384]
    assert local_segments(offs, 0, 384) == [0, 100, 384, 384]
    with pytest.raises(ValueError):
        shard_ranges(10, 0)


def _assembly_worker(rank, world, port, q, P, chunks):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from federatedscope_amd.core.sharding import PipelinedAssembly
        rng = np.random.default_rng(3)
        n = 5
        X = rng.standard_normal((n, P)).astype(np.float32)
        sizes = [int(s) for s in rng.integers(1, 100, n)]
        w = O.fedavg_weights(sizes)
        pa = PipelinedAssembly(P, chunks=chunks, align=16)
        seen = []

        def compute(j, lo, hi, view):
            seen.append((j, lo, hi))
            got = O.para_weighted_avg([(s, {'w': X[i, lo:hi]})
                                       for i, s in enumerate(sizes)],
                                      weights=w)['w']
            view.copy_(torch.from_numpy(got.copy()))

        full = pa.run(compute).numpy()
        want = O.para_weighted_avg([(s, {'w': X[i]})
                                    for i, s in enumerate(sizes)],
                                   weights=w)['w']
        q.put((rank, full.tobytes() == want.tobytes(), seen,
               pa.local_numel()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world,P,chunks', [(2, 1000, 3), (2, 37, 4),
                                            (2, 4096, 1), (4, 1000, 3),
                                            (8, 5003, 4), (8, 37, 2)])
def test_pipelined_assembly_world2(world, P, chunks):
    """Block-cyclic pieces + in-place all-gather per round reproduce the
    single-device FedAvg bit for bit, ragged tails and empty pieces
    included; every coordinate is computed by exactly one rank (world 2, and
    the 4- and 8-rank plans the driver's multi-GPU runs use)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_assembly_worker,
                         args=(r, world, port, q, P, chunks))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    assert all(r[1] for r in res), res
    covered = sorted((lo, hi) for r in res for _, lo, hi in r[2])
    pos = 0
    for lo, hi in covered:
        assert lo == pos
        pos = hi
    assert pos == P


def test_pipelined_assembly_stream_choice():
    """Pieces below SMALL_PIECE coordinates alternate over two side streams
    (one GPU's share at 8 GPUs); larger pieces, a single round or an
    explicit count keep what they are given."""
    from federatedscope_amd.core.sharding import PipelinedAssembly
    small = PipelinedAssembly(25_000_000 // 8, chunks=4)
    assert small.pc < PipelinedAssembly.SMALL_PIECE and small.streams == 2
    big = PipelinedAssembly(25_000_000 // 4, chunks=4)
    assert big.pc >= PipelinedAssembly.SMALL_PIECE and big.streams == 1
    assert PipelinedAssembly(1000, chunks=1).streams == 1
    assert PipelinedAssembly(1000, chunks=4, streams=3).streams == 3
    with pytest.raises(ValueError):
        PipelinedAssembly(1000, chunks=4, streams=0)


def test_pipelined_assembly_plan_world1():
    from federatedscope_amd.core.sharding import PipelinedAssembly
    pa = PipelinedAssembly(1000, chunks=3, align=64)
    assert pa.pc == 384 and pa.padded == 1152
    assert pa.local_pieces() == [(0, 384), (384, 768), (768, 1000)]
    out = pa.run(lambda j, lo, hi, v: v.copy_(torch.arange(lo, hi,
                                                           dtype=v.dtype)))
    assert torch.equal(out, torch.arange(1000, dtype=torch.float32))
    with pytest.raises(ValueError):
        PipelinedAssembly(10, chunks=0)


class _FakePeerLib:
    """The peer-memory entry points of libfsagg as host stand-ins, so that
    PeerAssembly's setup protocol runs without a GPU; ``deny`` makes this
    rank's fsagg_peer_can_access refuse a peer (a GPU without a link)."""

    def __init__(self, rank, deny):
        self.rank, self.deny, self.n = rank, deny, 0
        self.freed, self.closed = [], []

    def fsagg_peer_handle_bytes(self):
        return 8

    def fsagg_peer_alloc(self, dev, nbytes, out):
        self.n += 1
        out._obj.value = 0x1000 * (self.rank + 1) + self.n
        return 0

    def fsagg_peer_pci_bus_id(self, dev, buf, size):
        buf.value = b'0000:%02x:00.0' % self.rank
        return 0

    def fsagg_peer_can_access(self, dev, bus):
        return 0 if self.deny else 1

    def fsagg_peer_handle(self, ptr, buf):
        buf.raw = int(ptr).to_bytes(8, 'little')
        return 0

    def fsagg_peer_open(self, dev, buf, out):
        out._obj.value = int.from_bytes(buf.raw[:8], 'little') | 1 << 40
        return 0

    def fsagg_peer_close(self, dev, p):
        self.closed.append(p)

    def fsagg_peer_free(self, dev, p):
        self.freed.append(p)


def _peer_setup_worker(rank, world, port, deny_rank, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from federatedscope_amd import _lib as L
        from federatedscope_amd.core import sharding
        fake = _FakePeerLib(rank, rank == deny_rank)
        L.load = lambda: fake
        try:
            sharding.PeerAssembly(1000, device='cuda:0')
            q.put((rank, 'built', len(fake.freed)))
        except RuntimeError as e:
            # every allocation released, nothing left open
            q.put((rank, 'refused:' + str(e)[:40], len(fake.freed),
                   fake.n, len(fake.closed)))
        # the ranks are still in step: a collective after the refusal
        t = torch.ones(1)
        dist.all_reduce(t)
        q.put((rank, 'sum', float(t)))
    finally:
        dist.destroy_process_group()


def test_peer_assembly_setup_agrees_across_ranks():
    """One rank cannot reach a peer: every rank refuses the peer assembly
    (so all fall back to the collective together), every rank releases its
    allocations, and the ranks stay in step for the next collective."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_peer_setup_worker,
                      args=(r, world, port, 1, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in range(2 * world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    refused = sorted(o for o in out if o[1] != 'sum')
    assert [o[0] for o in refused] == [0, 1]
    for o in refused:
        assert o[1].startswith('refused:')
        assert o[2] == o[3]          # every allocation freed
    assert sorted(o[2] for o in out if o[1] == 'sum') == [2.0, 2.0]
