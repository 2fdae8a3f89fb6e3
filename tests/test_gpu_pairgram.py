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
* structured data where the k-steps' roundings do not cancel (DESIGN
  §3.3): dequantised int8-grid uploads, Student-t (ν = 3) tails, a
  colluding group shifted by one sign-biased offset away from the centre,
  half-zero sparse updates — keys of >= 1M coordinates.
Contract checked: every per-key |d²_got − d²_fp64| is within the kernel's
worst-case bound err; the unflagged pairs' per-key distances are within
_GRAM_TOL (1e-6) of fp64 (Σ_s |d_s − d̂_s| <= 1e-6 · Σ_s d_s), and D — the
reference's fp32 formation of them — within 1e-6 plus the fp32 rounding of
that formation."""
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


def _formation(nseg):
    """Relative slack between two fp32 formations of D (a per-key fl32 sqrt
    and an fp32 sum over nseg keys) from inputs that differ: one rounding
    step each may land on the other side."""
    return 2.0 * (nseg + 1) * 2.0 ** -24


def _check(got, err, D, flags, want, rtol=1e-6):
    """Returns max |d²_got − d²_fp64| / err over the keys and pairs."""
    # the worst-case bound holds on every key and pair
    dev = np.abs(got - want)
    assert np.all(dev <= err), np.max(dev / np.maximum(err, 1e-300))
    ratio = float(np.max(np.where(err > 0, dev / np.maximum(err, 1e-300),
                                  0.0)))
    # identical d² = 0 rows stay 0
    Dw = _fp64_D(want)
    off = ~np.eye(D.shape[0], dtype=bool) & ~flags
    pos = off & (Dw > 0)
    assert np.all(D[off & (Dw == 0)] == 0.0)
    if pos.any():
        # the certified per-key distances
        dk = np.abs(np.sqrt(got) - np.sqrt(want)).sum(0)
        sk = np.sqrt(want).sum(0)
        assert np.all(dk[pos] <= rtol * sk[pos] + 1e-300), \
            (dk[pos] / sk[pos]).max()
        e = np.abs(D[pos].astype(np.float64) - Dw[pos]) / Dw[pos]
        assert e.max() <= rtol + _formation(got.shape[0]), e.max()
    return ratio


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
        assert e.max() <= 1e-6 + _formation(len(lay.keys))
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
    assert err.max() <= 1e-6 + _formation(len(lay.keys))


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
        assert err.max() <= 1e-6 + _formation(1)


def _fp64_segsq_dev(clients, lay):
    """_fp64_segsq on the device (fp64 torch, direct differences): the
    stress keys hold >= 1M coordinates."""
    n = len(clients)
    out = np.zeros((len(lay.keys), n, n))
    for s, k in enumerate(lay.keys):
        X = torch.stack([c[k].reshape(-1) for c in clients]).double()
        sq = torch.empty((n, n), dtype=torch.float64, device=X.device)
        for a in range(n):
            sq[a] = ((X - X[a]) ** 2).sum(1)
        out[s] = sq.cpu().numpy()
    return out


STRESS_SIZES = [1_000_003, 4097, 33]


def _stress_clients(family, n=50, seed=123):
    """n clients of one structured data family:
    int8_grid   — dequantised int8 uploads: base + small noise quantised to
                  a per-client grid of max|x|/127 (most coordinates equal
                  across clients, the rest one grid step apart);
    student_t3  — base + heavy-tailed (ν = 3) noise;
    offset      — half the coordinates frozen (equal in every client), and
                  a colluding group of 10 shifted by one sign-biased offset
                  (+0.3 everywhere, frozen coordinates included) away from
                  the honest centre;
    sparse      — half-zero updates (independent masks)."""
    g = torch.Generator(device='cuda').manual_seed(seed)
    base = [torch.randn(sz, device='cuda', generator=g) for sz in
            STRESS_SIZES]
    frozen = [torch.rand(sz, device='cuda', generator=g) < 0.5 for sz in
              STRESS_SIZES]

    def fn(i, j, z):
        if family == 'int8_grid':
            y = base[j] + 0.01 * z
            sc = y.abs().max() / 127.0
            return torch.clamp(torch.round(y / sc), -127, 127) * sc
        if family == 'student_t3':
            c = sum(torch.randn(z.shape, device='cuda', generator=g) ** 2
                    for _ in range(3)) / 3.0
            return base[j] + 0.01 * z / c.sqrt()
        if family == 'offset':
            y = torch.where(frozen[j], base[j], base[j] + 0.01 * z)
            return y + 0.3 if i < 10 else y
        if family == 'sparse':
            keep = torch.rand(z.shape, device='cuda', generator=g) < 0.5
            return torch.where(keep, z, torch.zeros_like(z))
        raise ValueError(family)
    return _clients(n, sizes=STRESS_SIZES, seed=seed + 1, fn=fn)


@pytest.mark.parametrize('family', ['int8_grid', 'student_t3', 'offset',
                                    'sparse'])
def test_pairgram_stress_families(family):
    """Structured data, 50 clients, keys of 1M / 4097 / 33: the worst-case
    per-key bound holds on every pair, the pairs it leaves unflagged are
    certified to 1e-6, and the engine's D (flagged pairs recomputed on the
    VALU kernel) is within 1e-6 of fp64 with the fp64 selection."""
    import json
    import os
    from federatedscope_amd.core.aggregators.krum_aggregator import \
        krum_scores
    clients = _stress_clients(family)
    n = len(clients)
    lay, _, _, stacked = _sets(clients)
    want = _fp64_segsq_dev(clients, lay)
    got, err, D, flags = _gram(stacked)
    ratio = _check(got, err, D, flags, want)
    agg = _krum(clients, f=10)
    De, _ = agg.distance_matrix([(1, c) for c in _as_slab(clients)])
    assert agg.last_pairdist_path.startswith('mfma'), agg.last_pairdist_path
    Dw = _fp64_D(want)
    off = ~np.eye(n, dtype=bool)
    pos = off & (Dw > 0)
    rel = float((np.abs(De.numpy()[pos] - Dw[pos]) / Dw[pos]).max())
    assert rel <= 1e-6 + _formation(len(lay.keys)), rel
    s_ref = np.sort(Dw, axis=1)[:, :n - 10 - 2].sum(-1)
    order = np.argsort(s_ref, kind='stable')
    s_got = krum_scores(De, 10).numpy()
    srt = np.sort(s_ref)
    if (srt[1] - srt[0]) / srt[0] >= 1e-5:
        assert int(np.argmin(s_got)) == int(order[0])
    rec = {'family': family, 'max_abserr_over_bound': ratio,
           'flagged_pairs': int(flags.sum()) // 2,
           'engine_path': agg.last_pairdist_path,
           'engine_max_rel_err_vs_fp64': rel}
    log = os.environ.get('FSAGG_TEST_LOG')
    if log:
        with open(log, 'a') as fh:
            fh.write(json.dumps(rec) + '\n')
