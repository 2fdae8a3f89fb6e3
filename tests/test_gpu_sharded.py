"""Param-range sharded kernels on one GPU: every shard computed separately
(as rank g would) and stitched together must equal the unsharded result —
bit-exact for FedAvg / median, exact selection for Krum (the per-key
partials are summed across shards as the all-reduce would)."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


def _setup(n=9, P=12345, seed=5):
    from federatedscope_amd import ops
    from federatedscope_amd.core.sharding import shard_ranges
    dev = torch.device('cuda', 0)
    ld = ops.round_up(P, 64)
    slab = torch.empty((n, ld), device=dev)
    ops.fill_uniform(slab, P, seed=seed)
    return dev, slab, ld


@pytest.mark.parametrize('world', [1, 2, 3, 8])
def test_sharded_fedavg_median_bit_exact(world):
    from federatedscope_amd import ops
    from federatedscope_amd.core.sharding import shard_ranges
    n, P = 9, 100_003
    dev, slab, ld = _setup(n, P)
    w = O.fedavg_weights(list(range(1, n + 1)))
    full = torch.empty(P, device=dev)
    ops.weighted_sum(ops.RowTable.from_slab(slab, numel=P), w, full)
    fullmed = torch.empty(P, device=dev)
    ops.coord_median(ops.RowTable.from_slab(slab, numel=P), fullmed)
    out = torch.empty(P, device=dev)
    med = torch.empty(P, device=dev)
    for lo, hi in shard_ranges(P, world):
        if hi == lo:
            continue
        rows = ops.RowTable.from_slab(slab, col_offset=lo, numel=hi - lo)
        ops.weighted_sum(rows, w, out[lo:hi])
        ops.coord_median(rows, med[lo:hi])
    assert torch.equal(out, full)
    assert torch.equal(med, fullmed)
    # and against the oracle on the host
    X = slab[:, :P].cpu().numpy()
    want = O.para_weighted_avg([(1, {'w': X[i]}) for i in range(n)],
                               weights=w)['w']
    assert out.cpu().numpy().tobytes() == want.tobytes()


@pytest.mark.parametrize('world', [2, 4])
def test_sharded_krum_partials(world):
    from federatedscope_amd import ops
    from federatedscope_amd.core.sharding import local_segments, shard_ranges
    n, P = 12, 50_000
    dev, slab, ld = _setup(n, P, seed=9)
    offs = [0, 7, 20000, 20003, P]
    D1 = ops.pairdist(ops.RowTable.from_slab(slab, numel=P), offs)
    acc = None
    for lo, hi in shard_ranges(P, world):
        rows = ops.RowTable.from_slab(slab, col_offset=lo, numel=hi - lo)
        sq = ops.pairdist_segsq(rows, local_segments(offs, lo, hi))
        acc = sq if acc is None else acc + sq
    D2 = ops.pairdist_finish(acc)
    off = ~torch.eye(n, dtype=torch.bool, device=dev)
    assert torch.allclose(D1[off], D2[off], rtol=1e-6)
    X = slab[:, :P].cpu().numpy()
    paras = [{'k%d' % s: X[i, offs[s]:offs[s + 1]] for s in range(4)}
             for i in range(n)]
    Dref = O.krum_distance_matrix(paras)
    np.testing.assert_allclose(D2.cpu().numpy()[off.cpu().numpy()],
                               Dref[off.cpu().numpy()], rtol=1e-5)
    assert O.krum_select(O.krum_scores(D2.cpu().numpy(), 2), 4) == \
        O.krum_select(O.krum_scores(Dref, 2), 4)


@pytest.mark.parametrize('chunks', [1, 3, 8])
def test_pipelined_assembly_gpu_world1_bit_exact(chunks):
    """PipelinedAssembly's piece plan driving the FedAvg kernel (one rank:
    no collective) reproduces the unsharded result bit for bit."""
    from federatedscope_amd import ops
    from federatedscope_amd.core.sharding import PipelinedAssembly
    n, P = 7, 100_003
    dev, slab, ld = _setup(n, P)
    w = O.fedavg_weights(list(range(3, n + 3)))
    full = torch.empty(P, device=dev)
    ops.weighted_sum(ops.RowTable.from_slab(slab, numel=P), w, full)
    pa = PipelinedAssembly(P, chunks=chunks)

    def compute(j, lo, hi, view):
        ops.weighted_sum(ops.RowTable.from_slab(slab, col_offset=lo,
                                                numel=hi - lo), w, view)

    got = pa.run(compute, device=dev)
    assert torch.equal(got, full)


@pytest.mark.parametrize('world,rank,streams,split', [
    (4, 0, 1, None), (4, 3, 2, None), (8, 5, 2, 'taper'), (8, 0, 1, 'taper'),
    (2, 1, 2, (3, 1))])
def test_pipelined_assembly_async_comm_ordering(world, rank, streams, split):
    """PipelinedAssembly.run under a Comm whose all-gather returns a real
    async work handle (tools/emu_comm.py: the gather runs on its own stream,
    waits on the issuing stream and is delayed by a spin kernel, as RCCL's
    in-place all_gather_into_tensor(async_op=True) does).  The code path only
    RCCL reaches: works/w.wait() and the side-stream hand-off.  Every piece
    the collective read must be the finished piece, and the assembled result
    must be bit-exact once run() returns (read on the caller's stream)."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), 'tools'))
    from emu_comm import EmuComm
    from federatedscope_amd import ops
    from federatedscope_amd.core.sharding import (PipelinedAssembly,
                                                  tapered_split)
    n, P = 11, 1_000_003
    dev, slab, ld = _setup(n, P, seed=21)
    w = O.fedavg_weights(list(range(5, n + 5)))
    split = tapered_split(4) if split == 'taper' else split
    probe = EmuComm(world, rank, dev)
    pa = PipelinedAssembly(P, comm=probe, streams=streams, split=split)
    expected = torch.zeros(pa.padded, device=dev)
    ops.weighted_sum(ops.RowTable.from_slab(slab, numel=P), w,
                     expected[:P])
    out = torch.full((pa.padded, ), float('nan'), device=dev)
    comm = EmuComm(world, rank, dev, expected=expected, base=out,
                   delay_us=300.0)
    pa = PipelinedAssembly(P, comm=comm, streams=streams, split=split)
    assert pa.streams == streams

    def compute(j, lo, hi, view):
        # a slow piece: the spin makes a collective that does not wait for
        # its piece read NaNs
        torch.cuda._sleep(200_000)
        ops.weighted_sum(ops.RowTable.from_slab(slab, col_offset=lo,
                                                numel=hi - lo), w, view)

    torch.cuda.synchronize()
    got = pa.run(compute, out=out)
    # read on the caller's stream right away (no synchronize before it)
    res = got.clone()
    assert comm.calls == pa.chunks
    assert torch.equal(res, expected[:P])
    for j, (own, snap) in enumerate(sorted(comm.sent, key=lambda s: s[0])):
        lo, hi = pa.piece(j)
        assert own == pa.slot(j)
        assert torch.equal(snap[:hi - lo], expected[lo:hi])
