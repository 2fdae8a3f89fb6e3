"""Krum distances on the matrix cores (fsagg_pairgram_rows_segsq_f32 +
fsagg_pairgram_finish_f32).

The Gram form d² = G_aa + G_bb − 2·G_ab (centred on a central client, bf16
limbs, fp32 within a k-step / fp64 beyond) against an fp64 restatement of
every per-key squared distance, and against the VALU kernel (pairdist.hip):
* n = 2 … 64 (1–4 MFMA tiles, ragged last tile), keys of 0, 1, 3, 5 … 300k
  elements (partial k-steps, chunk tails), keyed and stacked row sets;
* rows that are not 16-B aligned (the per-element load path);
* a common component 1000× the spread (cancellation without centring),
  with a far Byzantine client;
* identical and near-duplicate clients far from the others (their pair
  flagged; the engine recomputes the flagged clients' pairs exactly on the
  VALU kernel), and non-finite values (flagged, VALU semantics).
Contract checked: every per-key |d²_got − d²_fp64| is within the kernel's
own predicted bound (err + 2e-8·d²); unflagged Krum distances D are within
_GRAM_TOL (1e-6) of fp64."""
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


def _as_slab(clients):
    """The same clients as views of one allocation (each client's keys
    contiguous, as in the client stack): rows at spread offsets, the layout
    the engine gives the matrix cores (_engine._rows_spread)."""
    keys = list(clients[0].keys())
    sizes = [clients[0][k].numel() for k in keys]
    total = sum(sizes) + 16 * len(keys)
    slab = torch.zeros((len(clients), total), device='cuda')
    out = []
    for i, c in enumerate(clients):
        d, o = OrderedDict(), 0
        for k, sz in zip(keys, sizes):
            d[k] = slab[i, o:o + sz].view(c[k].shape)
            d[k].copy_(c[k])
            o += (sz + 15) // 16 * 16
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
    """The Gram path over every key: (segsq, err, D, flags) on the host."""
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import _GRAM_TOL
    sq2 = ops.pairgram_rows_segsq(rs)
    _, D, ill = ops.pairgram_finish(sq2, _GRAM_TOL)
    flags = ill.cpu().numpy()
    sq2 = sq2.cpu().numpy()
    return sq2[0], sq2[1], D.cpu().numpy(), (flags + flags.T) > 0


def _fp64_D(want):
    """The reference's D (fp32 sum over keys of fp32 per-key distances),
    from fp64 per-key squared distances."""
    n = want.shape[1]
    D = np.zeros((n, n), dtype=np.float32)
    for s in range(want.shape[0]):
        D = (D + np.sqrt(want[s]).astype(np.float32)).astype(np.float32)
    np.fill_diagonal(D, np.inf)
    return D


# pairgram.hip kErrBias: the part of the error proportional to d²
_BIAS = 2e-8


def _check(got, err, D, flags, want, rtol=1e-6):
    # the predicted bound holds on every key and pair
    bound = err + _BIAS * want
    assert np.all(np.abs(got - want) <= bound + 1e-300), \
        np.max(np.abs(got - want) / (bound + 1e-300))
    # identical d² = 0 rows stay 0
    Dw = _fp64_D(want)
    off = ~np.eye(D.shape[0], dtype=bool) & ~flags
    pos = off & (Dw > 0)
    assert np.all(D[off & (Dw == 0)] == 0.0)
    if pos.any():
        e = np.abs(D[pos].astype(np.float64) - Dw[pos]) / Dw[pos]
        assert e.max() <= rtol, e.max()


@pytest.mark.parametrize('n', [2, 5, 16, 17, 33, 50, 64])
def test_pairgram_vs_fp64_and_valu(n):
    from federatedscope_amd import ops
    clients = _clients(n, seed=n)
    lay, _, keyed, stacked = _sets(clients)
    want = _fp64_segsq(clients, lay)
    for rs in (keyed, stacked):
        got, err, D, flags = _gram(rs)
        assert flags.sum() <= 2, flags.sum()
        _check(got, err, D, flags, want)
    valu = ops.pairdist_rows_segsq(keyed).cpu().numpy()
    d_got, d_want = np.sqrt(valu), np.sqrt(want)
    pos = d_want > 0
    assert np.all(d_got[~pos] == 0.0)
    assert (np.abs(d_got[pos] - d_want[pos]) / d_want[pos]).max() <= 2e-7


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
    got, err, D, flags = _gram(rs)
    assert not flags.any()
    _check(got, err, D, flags, _fp64_segsq(clients, lay))


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
    got, err, D, flags = _gram(keyed)
    assert not flags.any()
    _check(got, err, D, flags, _fp64_segsq(clients, lay))


def _krum(clients, f=2):
    from types import SimpleNamespace
    from federatedscope_amd.core.aggregators import KrumAggregator
    cfg = SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=1000, sample_client_rate=1.0),
        aggregator=SimpleNamespace(
            byzantine_node_num=f,
            BFT_args=SimpleNamespace(krum_agg_num=1)))
    return KrumAggregator(device='cuda', config=cfg)


@pytest.mark.parametrize('case', ['identical', 'near', 'nonfinite'])
def test_pairgram_flags_and_exact_repair(case):
    n = 24

    def fn(i, j, z):
        if i in (3, 4):
            if case == 'identical':
                return torch.full_like(z, 50.0)
            return 50.0 + 1e-6 * z
        if case == 'nonfinite' and i == 9 and j == 0:
            z = z.clone()
            z[17] = float('inf')
        return z

    clients = _clients(n, sizes=[10_000, 33], seed=6, fn=fn)
    lay, _, keyed, _ = _sets(clients)
    got, err, D, flags = _gram(keyed)
    want = _fp64_segsq(clients, lay)
    if case == 'nonfinite':
        assert flags[9].sum() == n - 1
    else:
        assert flags[3, 4]
        assert flags.sum() <= 2 * (2 * n - 3)
        assert got[:, 3, 4].max() == 0.0 or case == 'near'
        _check(got, err, D, flags, want)
    agg = _krum(clients)
    De, _ = agg.distance_matrix([(1, c) for c in _as_slab(clients)])
    assert agg.last_pairdist_path.startswith('mfma + exact')
    # the recomputed pairs are the VALU kernel's (its semantics for ±inf)
    from federatedscope_amd import ops
    Dv = ops.pairdist_finish(ops.pairdist_rows_segsq(keyed)).cpu().numpy()
    sel = sorted(set(np.nonzero(flags)[0].tolist()))
    ix = np.ix_(sel, sel)
    assert np.allclose(De.numpy()[ix], Dv[ix], rtol=2e-7, atol=0,
                       equal_nan=True)
    if case != 'nonfinite':
        Dw = _fp64_D(want)
        off = ~np.eye(n, dtype=bool)
        pos = off & (Dw > 0)
        e = np.abs(De.numpy()[pos] - Dw[pos]) / Dw[pos]
        assert e.max() <= 1e-6
        assert De.numpy()[3, 4] == Dw[3, 4] or case == 'near'


@pytest.mark.parametrize('n', [7, 50])
def test_krum_distance_matrix_engine(n):
    """Through the engine: every key on the matrix cores, one distance
    matrix within 1e-6 of fp64 (summed over keys in fp32 like the
    reference), no pair recomputed."""
    clients = _clients(n, seed=40 + n)
    lay = _sets(clients)[0]
    agg = _krum(clients, f=1)
    D, _ = agg.distance_matrix([(1, c) for c in _as_slab(clients)])
    assert agg.last_pairdist_path == 'mfma'
    Dw = _fp64_D(_fp64_segsq(clients, lay))
    off = ~np.eye(n, dtype=bool)
    err = np.abs(D.numpy()[off] - Dw[off]) / Dw[off]
    assert err.max() <= 1e-6


def test_krum_distance_path_by_row_placement():
    """Rows that all start at one offset within a 2 MiB page (separately
    allocated 2 MiB-aligned tensors) take the VALU kernel, rows of one
    allocation the matrix cores; both within 1e-6 of fp64."""
    n = 12
    m = 600_000
    stride = 1 << 20                 # floats: rows 4 MiB apart
    g = torch.Generator(device='cuda').manual_seed(77)
    big = torch.randn((n, stride), device='cuda', generator=g)
    sep = [OrderedDict(w=big[i, :m]) for i in range(n)]
    assert len({c['w'].data_ptr() % (1 << 21) for c in sep}) == 1
    lay = _sets(sep)[0]
    Dw = _fp64_D(_fp64_segsq(sep, lay))
    off = ~np.eye(n, dtype=bool)
    for clients, path in ((sep, 'valu'), (_as_slab(sep), 'mfma')):
        agg = _krum(clients, f=1)
        D, _ = agg.distance_matrix([(1, c) for c in clients])
        assert agg.last_pairdist_path == path
        err = np.abs(D.numpy()[off] - Dw[off]) / Dw[off]
        assert err.max() <= 1e-6
