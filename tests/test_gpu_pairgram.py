"""Krum distances on the matrix cores (fsagg_pairgram_rows_segsq_f32).

The Gram form d² = G_aa + G_bb − 2·G_ab (centred on a central client, bf16
limbs, fp32-within-4-k-steps / fp64 accumulation) against an fp64
restatement of every per-key squared distance, and against the VALU
kernel (pairdist.hip):
* n = 2 … 64 (1–4 MFMA tiles, ragged last tile), keys of 0, 1, 3, 5 … 300k
  elements (partial k-steps, chunk tails), keyed and stacked row sets;
* rows that are not 16-B aligned (the per-element load path);
* a common component 1000× the spread (cancellation without centring),
  with a far Byzantine client;
* identical clients (d = 0 exactly, no flag) and near-duplicates far from
  the others (their pair flagged; the engine recomputes the flagged
  clients' pairs exactly on the VALU kernel).
Tolerance: 2e-7 relative on each per-key distance (the VALU kernel's
measured error is 1.6e-7 on C4)."""
from collections import OrderedDict

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [1, 0, 1023, 5, 300_001, 3, 7, 65_537, 33, 16]


def _clients(n, sizes=SIZES, seed=9, fn=None):
    g = torch.Generator(device='cuda').manual_seed(seed)
    out = []
    for i in range(n):
        d = OrderedDict()
        for j, sz in enumerate(sizes):
            z = torch.randn(sz, device='cuda', generator=g)
            d['k%d' % j] = fn(i, j, z) if fn else z
        out.append(d)
    return out


def _sets(clients):
    from federatedscope_amd import ops
    from federatedscope_amd.layout import BucketLayout, ClientStack
    lay = BucketLayout(OrderedDict((k, v.cpu()) for k, v in
                                   clients[0].items()))
    st = ClientStack(lay, len(clients), 'cuda')
    st.slab.zero_()
    st.load_many(clients)
    ptrs = np.array([[c[k].data_ptr() for k in lay.keys] for c in clients],
                    dtype=np.int64)
    keyed = ops.RowSet.from_pointers(lay, ptrs, 'cuda', keepalive=clients)
    stacked = ops.RowSet.from_stack(st, range(len(clients)))
    return lay, st, keyed, stacked


def _fp64_segsq(clients, lay):
    n = len(clients)
    out = np.zeros((len(lay.keys), n, n))
    for s, k in enumerate(lay.keys):
        X = np.stack([c[k].double().cpu().numpy().ravel() for c in clients])
        for a in range(n):
            out[s, a] = ((X - X[a]) ** 2).sum(axis=1)
    return out


def _gram(rs):
    """The Gram path over the keys the engine gives it (>= 4096 elements);
    returns (segsq, ill, mask of those keys)."""
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import _gram_key
    ill = torch.zeros((rs.n, rs.n), dtype=torch.int32, device='cuda')
    sq = ops.pairgram_rows_segsq(rs, ill, keep=_gram_key)
    big = np.array([_gram_key(rs.layout.numels[k]) for k in rs.layout.keys])
    got = sq.cpu().numpy()
    assert np.all(got[~big] == 0.0)
    flags = ill.cpu().numpy()
    return got[big], (flags + flags.T) > 0, big


def _check(got, want, rtol=2e-7):
    d_got, d_want = np.sqrt(got), np.sqrt(want)
    pos = d_want > 0
    assert np.all(d_got[~pos] == 0.0)
    err = np.abs(d_got[pos] - d_want[pos]) / d_want[pos]
    assert err.max() <= rtol, err.max()


@pytest.mark.parametrize('n', [2, 5, 16, 17, 33, 50, 64])
def test_pairgram_vs_fp64_and_valu(n):
    from federatedscope_amd import ops
    clients = _clients(n, seed=n)
    lay, _, keyed, stacked = _sets(clients)
    want = _fp64_segsq(clients, lay)
    for rs in (keyed, stacked):
        got, ill, big = _gram(rs)
        assert not ill.any()
        _check(got, want[big])
    valu = ops.pairdist_rows_segsq(keyed).cpu().numpy()
    _check(valu, want)


def test_pairgram_unaligned_rows():
    """Key tensors at 4-B offsets: the per-element load path."""
    from federatedscope_amd import ops
    from federatedscope_amd.layout import BucketLayout
    n = 20
    base = _clients(n, sizes=[4099, 77, 1_000_003], seed=3)
    clients = [OrderedDict((k, torch.cat([v[:1], v])[1:]) for k, v in
                           c.items()) for c in base]
    assert any(c['k0'].data_ptr() % 16 for c in clients)
    lay = BucketLayout(OrderedDict((k, v.cpu()) for k, v in
                                   clients[0].items()))
    ptrs = np.array([[c[k].data_ptr() for k in lay.keys] for c in clients],
                    dtype=np.int64)
    rs = ops.RowSet.from_pointers(lay, ptrs, 'cuda', keepalive=clients,
                                  aligned16=False)
    got, ill, big = _gram(rs)
    assert not ill.any()
    _check(got, _fp64_segsq(clients, lay)[big])


def test_pairgram_common_component_and_byzantine():
    """Updates = a shared vector 1000× their spread (the Gram form without
    centring would lose ~6 digits), one client 100× farther out."""
    n = 40
    g = torch.Generator(device='cuda').manual_seed(11)
    common = [torch.randn(sz, device='cuda', generator=g)
              for sz in [300_001, 4097, 9]]

    def fn(i, j, z):
        v = common[j] + 1e-3 * z
        return v + 0.1 * torch.ones_like(v) if i == 7 else v

    clients = _clients(n, sizes=[300_001, 4097, 9], seed=12, fn=fn)
    lay, _, keyed, _ = _sets(clients)
    got, ill, big = _gram(keyed)
    assert not ill.any()
    _check(got, _fp64_segsq(clients, lay)[big], rtol=1e-6)


def test_pairgram_duplicates_and_fallback():
    from types import SimpleNamespace
    from federatedscope_amd.core.aggregators import KrumAggregator
    n = 24

    def dup(i, j, z):
        # clients 3 and 4 identical, far from the rest
        return torch.full_like(z, 50.0) if i in (3, 4) else z

    clients = _clients(n, sizes=[10_000, 33], seed=5, fn=dup)
    lay, _, keyed, _ = _sets(clients)
    got, ill, big = _gram(keyed)
    assert got[:, 3, 4].max() == 0.0 and not ill.any()
    _check(got, _fp64_segsq(clients, lay)[big])

    # near-duplicates far from the centre: flagged, and the engine
    # recomputes with the VALU kernel
    def near(i, j, z):
        if i in (3, 4):
            return 50.0 + 1e-6 * z
        return z

    clients = _clients(n, sizes=[10_000, 33], seed=6, fn=near)
    lay, _, keyed, _ = _sets(clients)
    _, ill, _ = _gram(keyed)
    assert ill[3, 4] and ill.sum() <= 2 * (2 * n - 3)
    cfg = SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=1000, sample_client_rate=1.0),
        aggregator=SimpleNamespace(
            byzantine_node_num=2,
            BFT_args=SimpleNamespace(krum_agg_num=1)))

    class M(torch.nn.Module):
        def state_dict(self, *a, **kw):
            return OrderedDict((k, torch.zeros_like(v)) for k, v in
                               clients[0].items())

    agg = KrumAggregator(model=M(), device='cuda', config=cfg)
    D, _ = agg.distance_matrix([(1, c) for c in clients])
    assert agg.last_pairdist_path.startswith('mfma + exact')
    want = np.sqrt(_fp64_segsq(clients, lay)).sum(axis=0)
    off = ~np.eye(n, dtype=bool)
    err = np.abs(D.numpy()[off] - want[off]) / want[off]
    assert err.max() <= 2e-6


@pytest.mark.parametrize('n', [7, 50])
def test_krum_distance_matrix_mixed_keys(n):
    """Through the engine: big keys on the matrix cores, small keys on the
    VALU kernel, one distance matrix; within 2e-7 of fp64 (summed over
    keys in fp32 like the reference)."""
    from types import SimpleNamespace
    from federatedscope_amd.core.aggregators import KrumAggregator
    clients = _clients(n, seed=40 + n)
    lay = _sets(clients)[0]
    cfg = SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=1000, sample_client_rate=1.0),
        aggregator=SimpleNamespace(
            byzantine_node_num=1,
            BFT_args=SimpleNamespace(krum_agg_num=1)))
    agg = KrumAggregator(device='cuda', config=cfg)
    D, _ = agg.distance_matrix([(1, c) for c in clients])
    assert agg.last_pairdist_path == 'mfma'
    want = np.sqrt(_fp64_segsq(clients, lay)).sum(axis=0)
    off = ~np.eye(n, dtype=bool)
    err = np.abs(D.numpy()[off] - want[off]) / want[off]
    assert err.max() <= 1e-6
