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
