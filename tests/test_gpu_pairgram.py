"""Krum distances on the matrix cores (fsagg_pairgram_rows_segsq_f32 +
fsagg_pairgram_finish_f32, fsagg_pairgram_rows_f32).

The Gram form d² = G_aa + G_bb − 2·G_ab (centred on a central client, fp32
split exactly into three bf16 limbs, fp32 within an MFMA k-step / fp64
beyond) against an fp64 restatement of every per-key squared distance, and
against the VALU kernel (pairdist.hip):
* n = 2 … 64 (1–4 MFMA tiles, ragged last tile), keys of 0, 1, 3, 5 … 300k
  elements (partial k-steps, chunk tails), keyed and stacked row sets;
* rows that are not 16-B aligned (the per-element load path);
* a common component 1000× the spread (cancellation without centring),
  with a far Byzantine client;
* identical and near-duplicate clients far from the others, and non-finite
  values (flagged, recomputed with the VALU kernel's semantics);
* structured data where the k-steps' roundings do not cancel (DESIGN
  §3.3): dequantised int8-grid uploads, Student-t (ν = 3) tails, a
  colluding group shifted by one sign-biased offset away from the centre,
  half-zero sparse updates — keys of >= 1M coordinates.
Contract checked: every per-key |d²_got − d²_fp64| is within the kernel's
worst-case bound err; every finite pair's D is within its bound B (plus the
fp32 rounding of D's formation) of the fp64 distances' D; and the engine's
Krum selection — certified against B, else recomputed on the VALU kernel —
is the fp64 distances' selection wherever the fp64 scores separate it by
more than their own fp32 formation."""
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
    contiguous, as in the client stack)."""
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
    """The Gram path over every key: (segsq, err, D, flags, B) on the host."""
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import _GRAM_TOL
    sq2 = ops.pairgram_rows_segsq(rs)
    _, D, ill, B, _ = ops.pairgram_finish(sq2, _GRAM_TOL)
    flags = ill.cpu().numpy()
    sq2 = sq2.cpu().numpy()
    B = B.cpu().numpy().astype(np.float64)
    return sq2[0], sq2[1], D.cpu().numpy(), (flags + flags.T) > 0, \
        np.maximum(B, B.T)


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


def _check(got, err, D, flags, B, want):
    """Returns (max |d²_got − d²_fp64| / err, max |D − D_fp64| / B)."""
    # the worst-case bound holds on every key and pair
    dev = np.abs(got - want)
    assert np.all(dev <= err), np.max(dev / np.maximum(err, 1e-300))
    ratio = float(np.max(np.where(err > 0, dev / np.maximum(err, 1e-300),
                                  0.0)))
    # identical rows: d² = 0 exactly
    Dw = _fp64_D(want)
    off = ~np.eye(D.shape[0], dtype=bool) & ~flags
    assert np.all(D[off & (Dw == 0)] == 0.0)
    # the per-pair bound on D (a sum of per-key distances)
    dk = np.abs(np.sqrt(got) - np.sqrt(want)).sum(0)
    assert np.all(dk[off] <= B[off] * (1 + 1e-6) + 1e-300), \
        (dk[off] / np.maximum(B[off], 1e-300)).max()
    e = np.abs(D[off].astype(np.float64) - Dw[off].astype(np.float64))
    slack = _formation(got.shape[0]) * Dw[off].astype(np.float64)
    assert np.all(e <= B[off] + slack), (e - B[off] - slack).max()
    bratio = float(np.max(np.where(B[off] > 0, dk[off] / np.maximum(
        B[off], 1e-300), 0.0))) if off.any() else 0.0
    return ratio, bratio


def _separated(s, m, ordered, n):
    """Whether fp64-derived scores s fix the selection of m (and with
    ``ordered`` its order) beyond their own fp32 formation."""
    o = np.argsort(s, kind='stable')
    ss = s[o]
    gaps = range(min(m, len(s) - 1)) if ordered else [m - 1]
    return all(ss[i + 1] - ss[i] > 4 * n * 2.0 ** -23 * ss[i + 1]
               for i in gaps)


@pytest.mark.parametrize('n', [2, 5, 16, 17, 33, 50, 64, 65, 80, 100, 112,
                               120, 129, 200, 208, 209, 224, 241, 256])
def test_pairgram_vs_fp64_and_valu(n):
    """n <= 112: one workgroup forms every tile pair (65, 80, 100, 112:
    5..7 tiles, one workgroup per CU above 64); one 8-tile workgroup per
    chunk up to 128 clients (120); all 13 tiles on 16 waves up to 208 (129,
    200, 208); six 8-tile workgroups per chunk up to 256 (209, 224, 241,
    256: 14-16 tiles, absent tiles in the last groups) — with a last tile of
    1 client at 65, 129, 209 and 241."""
    from federatedscope_amd import ops
    clients = _clients(n, seed=n)
    lay, _, keyed, stacked = _sets(clients)
    want = _fp64_segsq(clients, lay) if n <= 64 else \
        _fp64_segsq_dev(clients, lay)
    for rs in (keyed, stacked):
        got, err, D, flags, B = _gram(rs)
        assert not flags.any()
        _check(got, err, D, flags, B, want)
    valu = ops.pairdist_rows_segsq(keyed).cpu().numpy()
    d_got, d_want = np.sqrt(valu), np.sqrt(want)
    pos = d_want > 0
    assert np.all(d_got[~pos] == 0.0)
    # the VALU kernel's fp32 in-stage sums (longer at larger n): measured
    # 2.2e-7 at n = 80, 4.2e-7 at 129, 9.5e-7 at 208
    tol = 2e-7 if n <= 64 else 1.5e-6 if n <= 208 else 3e-6
    assert (np.abs(d_got[pos] - d_want[pos]) / d_want[pos]).max() <= tol


@pytest.mark.parametrize('setting', [0, 2, 3])
@pytest.mark.parametrize('n', [65, 90, 100, 128, 150, 230])
def test_pairgram_workgroup_settings(setting, n):
    """Every n > 64 workgroup form of the A/B hook
    (fsagg_pairgram_set_block8): 0 the projective-plane lines, 2 four
    8-tile workgroups per chunk above 128 clients, 3 one workgroup holding
    every tile up to 128 (the default stops at 112) — each within the
    worst-case bounds of the fp64 distances."""
    from federatedscope_amd import _lib as L
    clients = _clients(n, seed=n + 1)
    lay, _, keyed, _ = _sets(clients)
    want = _fp64_segsq_dev(clients, lay)
    lib = L.load()
    prev = lib.fsagg_pairgram_set_block8(setting)
    try:
        got, err, D, flags, B = _gram(keyed)
    finally:
        lib.fsagg_pairgram_set_block8(prev)
    assert not flags.any()
    _check(got, err, D, flags, B, want)


@pytest.mark.parametrize('n', [2, 17, 31, 33, 49, 50, 52, 53, 64, 65, 100,
                               104, 105, 112])
def test_pairgram_compact_stages(n):
    """The compact stage buffers (the n client rows, three buffers where
    they fit: two stages in flight; fsagg_pairgram_set_stages 1) and the
    same with early release (2: every buffer's stage in flight under the
    compute) against the round-5 full-tile stages (0) on the same rows:
    every Gram sum is formed in the same order, so the per-key d², bounds
    and distances are identical bit for bit — both for keyed (separately
    allocated) and stacked rows — and within the fp64 distances' bounds."""
    from federatedscope_amd import _lib as L
    clients = _clients(n, sizes=[70_001, 4097, 33, 1_000_000], seed=n + 7)
    lay, _, keyed, stacked = _sets(clients)
    lib = L.load()
    res = {}
    for mode in (0, 1, 2, 3, 4):
        prev = lib.fsagg_pairgram_set_stages(mode)
        try:
            res[mode] = [_gram(keyed), _gram(stacked)]
        finally:
            lib.fsagg_pairgram_set_stages(prev)
    for m in (1, 2, 3, 4):
        for a, b in zip(res[0], res[m]):
            for x, y in zip(a, b):
                assert np.asarray(x).tobytes() == np.asarray(y).tobytes(), \
                    (n, m)
    got, err, D, flags, B = res[1][0]
    assert not flags.any()
    _check(got, err, D, flags, B, _fp64_segsq_dev(clients, lay))


@pytest.mark.parametrize('n', [2, 17, 50, 64, 65, 100, 129, 200, 256])
def test_pairgram_fused_tail(n):
    """The fused chain tail (fsagg_pairgram_set_fused 1, the default: the
    centre picked by the last pair-sum workgroup, each key's d² + bounds +
    the finish in one launch whose last workgroup per tile pair finishes
    it) against the round-5 eight-launch chain (0) on the same rows, keyed
    and stacked: the same sums in the same order, so d², bounds, D, flags
    and B are identical bit for bit."""
    from federatedscope_amd import _lib as L
    clients = _clients(n, sizes=[70_001, 4097, 33, 1_000_000] if n <= 100
                       else [4097, 33, 200_003], seed=n + 11)
    lay, _, keyed, stacked = _sets(clients)
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import _GRAM_TOL
    lib = L.load()

    def chain(rs):
        # the whole chain with its finish (fsagg_pairgram_rows_f32): buf =
        # D64, D, ill, B; sq2 = every key's d² and bound
        out = ops.pairgram_rows_dist(rs, _GRAM_TOL)
        return [out[0].cpu().numpy(), out[5].cpu().numpy()]
    res = {}
    for mode in (0, 1):
        prev = lib.fsagg_pairgram_set_fused(mode)
        try:
            res[mode] = [_gram(keyed), _gram(stacked), _gram(keyed),
                         chain(keyed), chain(stacked)]
        finally:
            lib.fsagg_pairgram_set_fused(prev)
    for a, b in zip(res[0], res[1]):
        for x, y in zip(a, b):
            assert np.asarray(x).tobytes() == np.asarray(y).tobytes(), n
    for x, y in zip(res[1][0], res[1][2]):
        assert np.asarray(x).tobytes() == np.asarray(y).tobytes(), n
    got, err, D, flags, B = res[1][0]
    assert not flags.any()
    _check(got, err, D, flags, B, _fp64_segsq_dev(clients, lay))


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
    got, err, D, flags, B = _gram(rs)
    assert not flags.any()
    _check(got, err, D, flags, B, _fp64_segsq(clients, lay))


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
    got, err, D, flags, B = _gram(keyed)
    assert not flags.any()
    _check(got, err, D, flags, B, _fp64_segsq(clients, lay))


def _krum(clients, f=2, m=1):
    from types import SimpleNamespace
    from federatedscope_amd.core.aggregators import KrumAggregator
    cfg = SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=1000, sample_client_rate=1.0),
        aggregator=SimpleNamespace(
            byzantine_node_num=f,
            BFT_args=SimpleNamespace(krum_agg_num=m)))
    return KrumAggregator(device='cuda', config=cfg)


class _DictModel(torch.nn.Module):
    def __init__(self, sd):
        super().__init__()
        self.sd = sd

    def state_dict(self, *a, **kw):
        return self.sd


def _select(clients, f, m):
    """The engine's Krum selection (KrumAggregator.aggregate on the clients
    as slab views, a zero init model) and its distance path."""
    agg = _krum(clients, f=f, m=m)
    agg.model = _DictModel(OrderedDict(
        (k, torch.zeros_like(v)) for k, v in clients[0].items()))
    agg.aggregate({'client_feedback': [(1, c) for c in _as_slab(clients)],
                   'recover_fun': None})
    return agg.last_selection, agg.last_pairdist_path


def _fp64_selection(want, f, m):
    from federatedscope_amd.core.aggregators.krum_aggregator import \
        krum_scores
    Dw = _fp64_D(want)
    n = Dw.shape[0]
    s = krum_scores(torch.from_numpy(Dw), f).double().numpy()
    return [int(i) for i in np.argsort(s, kind='stable')[:m]], \
        _separated(s, m, True, n)


@pytest.mark.parametrize('case', ['identical', 'near', 'nonfinite'])
def test_pairgram_flags_and_exact_repair(case):
    """Identical / near-duplicate clients far from the rest: bounded like
    every pair, no recomputation; a non-finite value: its client's pairs
    flagged and recomputed on the VALU kernel (its ±inf semantics)."""
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
    got, err, D, flags, B = _gram(keyed)
    want = _fp64_segsq(clients, lay)
    agg = _krum(clients)
    De, _ = agg.distance_matrix([(1, c) for c in _as_slab(clients)])
    if case == 'nonfinite':
        assert flags[9].sum() == n - 1
        assert agg.last_pairdist_path.startswith('mfma + exact')
        from federatedscope_amd import ops
        Dv = ops.pairdist_finish(ops.pairdist_rows_segsq(keyed)).cpu().numpy()
        sel = sorted(set(np.nonzero(flags)[0].tolist()))
        ix = np.ix_(sel, sel)
        assert np.allclose(De.numpy()[ix], Dv[ix], rtol=2e-7, atol=0,
                           equal_nan=True)
        # the recomputed pairs carry the VALU kernel's own bound: its fp32
        # per-chunk sums of at most chunk + 256 non-negative terms, halved
        # by the sqrt, plus D's own fp32 formation
        import math
        Dr = De.numpy()[ix].astype(np.float64)
        nseg = len(lay.keys)
        u = 2.0 ** -24
        chl = ops.L.load().fsagg_pairdist_chunk_elems(len(sel), lay.numel,
                                                      nseg)
        assert chl >= 2048
        acc = math.expm1((chl + 256) * math.log1p(u)) + 64 * u
        rel = acc / (2.0 * (1.0 - acc))
        want_b = (rel + (2 * nseg + 2) * u) * np.where(np.isfinite(Dr), Dr,
                                                        0.0)
        assert np.allclose(agg.last_pair_bound[ix], want_b, rtol=1e-12,
                           atol=0)
        # and it holds: |D − Σ_key sqrt(exact d²)| on the finite pairs
        with np.errstate(invalid='ignore'):
            exact = np.sqrt(want).sum(0)[ix]
        fin = np.isfinite(Dr) & np.isfinite(exact) & (Dr > 0)
        assert (np.abs(Dr - exact)[fin] <= agg.last_pair_bound[ix][fin]).all()
        return
    assert not flags.any()
    assert agg.last_pairdist_path == 'mfma'
    _check(got, err, D, flags, B, want)
    if case == 'identical':
        assert got[:, 3, 4].max() == 0.0 and De.numpy()[3, 4] == 0.0
    sel, path = _select(clients, f=2, m=3)
    want_sel, sep = _fp64_selection(want, 2, 3)
    if sep:
        assert sel == want_sel, (sel, want_sel, path)


@pytest.mark.parametrize('n', [7, 50])
def test_krum_distance_matrix_engine(n):
    """Through the engine: every key on the matrix cores, D within its
    per-pair bound of the fp64 distances, no pair recomputed, and the
    multi-Krum selection the fp64 one."""
    clients = _clients(n, seed=40 + n)
    lay = _sets(clients)[0]
    agg = _krum(clients, f=1)
    D, _ = agg.distance_matrix([(1, c) for c in _as_slab(clients)])
    assert agg.last_pairdist_path == 'mfma'
    want = _fp64_segsq(clients, lay)
    Dw = _fp64_D(want)
    off = ~np.eye(n, dtype=bool)
    B = agg.last_pair_bound
    e = np.abs(D.numpy()[off].astype(np.float64) - Dw[off])
    assert np.all(e <= B[off] + _formation(len(lay.keys)) * Dw[off])
    m = max(1, n // 3)
    sel, path = _select(clients, f=1, m=m)
    want_sel, sep = _fp64_selection(want, 1, m)
    if sep:
        assert sel == want_sel, (sel, want_sel, path)


def test_krum_distance_path_by_row_placement():
    """Rows of separately allocated 2 MiB-aligned tensors (the Gram kernel
    stages them through LDS) and rows of one allocation: both on the matrix
    cores, within their bounds of fp64."""
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
    for clients in (sep, _as_slab(sep)):
        agg = _krum(clients, f=1)
        D, _ = agg.distance_matrix([(1, c) for c in clients])
        assert agg.last_pairdist_path == 'mfma'
        B = agg.last_pair_bound
        e = np.abs(D.numpy()[off].astype(np.float64) - Dw[off])
        assert np.all(e <= B[off] + _formation(1) * Dw[off])


@pytest.mark.parametrize('n', [100, 200, 256])
def test_krum_engine_large_n(n):
    """Krum through the engine at n = 100 / 200 / 256: D within
    its per-pair bound of fp64, the multi-Krum selection the fp64 one."""
    f, m = n // 5, 5
    sizes = [400_003, 4097, 33]
    g = torch.Generator(device='cuda').manual_seed(500 + n)
    base = [torch.randn(sz, device='cuda', generator=g) for sz in sizes]

    def fn(i, j, z):
        if i % 9 == 4:                    # a Byzantine cluster
            return 0.1 + 0.05 * z
        return base[j] + 0.01 * (1 + 0.05 * (i % 13)) * z

    clients = _clients(n, sizes=sizes, seed=600 + n, fn=fn)
    lay = _sets(clients)[0]
    want = _fp64_segsq_dev(clients, lay)
    agg = _krum(clients, f=f)
    D, _ = agg.distance_matrix([(1, c) for c in _as_slab(clients)])
    assert agg.last_pairdist_path == 'mfma', agg.last_pairdist_path
    Dw = _fp64_D(want)
    off = ~np.eye(n, dtype=bool)
    B = agg.last_pair_bound
    e = np.abs(D.numpy()[off].astype(np.float64) - Dw[off])
    assert np.all(e <= B[off] + _formation(len(lay.keys)) * Dw[off])
    assert np.allclose(D.numpy(), D.numpy().T, rtol=0, atol=0)
    sel, path = _select(clients, f=f, m=m)
    want_sel, sep = _fp64_selection(want, f, m)
    assert path.startswith('mfma'), path
    if sep:
        assert sel == want_sel, (sel, want_sel, path)


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
    per-key bound and the per-pair bound on D hold on every pair, nothing is
    flagged, and the engine's multi-Krum selection (certified, else
    recomputed on the VALU kernel) is the fp64 one."""
    import json
    import os
    clients = _stress_clients(family)
    n = len(clients)
    f, m = 10, 5
    lay, _, _, stacked = _sets(clients)
    want = _fp64_segsq_dev(clients, lay)
    got, err, D, flags, B = _gram(stacked)
    assert not flags.any()
    ratio, bratio = _check(got, err, D, flags, B, want)
    sel, path = _select(clients, f=f, m=m)
    assert path.startswith('mfma'), path
    want_sel, sep = _fp64_selection(want, f, m)
    if sep:
        assert sel == want_sel, (sel, want_sel, path)
    Dw = _fp64_D(want)
    off = ~np.eye(n, dtype=bool)
    rel = float((np.abs(D[off].astype(np.float64) - Dw[off]) /
                 Dw[off]).max())
    brel = float((B[off] / Dw[off]).max())
    rec = {'family': family, 'max_abserr_over_bound_per_key': ratio,
           'max_D_err_over_pair_bound': bratio,
           'max_rel_err_D_vs_fp64': rel, 'max_rel_pair_bound': brel,
           'engine_path': path, 'fp64_selection_separated': sep}
    log = os.environ.get('FSAGG_TEST_LOG')
    if log:
        with open(log, 'a') as fh:
            fh.write(json.dumps(rec) + '\n')


def test_pairgram_graph_fresh_tables():
    """The captured chain (ops.pairgram_rows_dist_graph: one graph per
    shape whose first kernel fetches the row table from a pinned buffer
    the host refills per call) over three client sets of one shape at
    different addresses, in alternation and back to back without a
    synchronize between the calls: every call's buffer is bit-identical to
    the eager chain on the same rows."""
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import _GRAM_TOL
    sets = []
    for seed in (1, 2, 3):
        clients = _clients(37, sizes=[4097, 33, 70_001], seed=seed)
        sets.append(_sets(clients)[2])
    want = [ops.pairgram_rows_dist(rs, _GRAM_TOL)[0].cpu().numpy()
            for rs in sets]
    got = []
    for i in (0, 1, 2, 1, 0, 2, 2, 0):
        buf = ops.pairgram_rows_dist_graph(sets[i], _GRAM_TOL)[0]
        got.append((i, buf.to('cpu', non_blocking=False).numpy().copy()))
    for i, g in got:
        assert g.tobytes() == want[i].tobytes(), i


def test_pairgram_graph_cache_eviction():
    """More captured shapes than the cache holds: every call's buffer still
    matches the eager chain (evicted entries wait for their last replay's
    pinned-table fetch before their buffers are released)."""
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import _GRAM_TOL
    cap = ops._GraphCache.MAX_ENTRIES
    sets = []
    for j in range(cap + 3):
        clients = _clients(3 + j, sizes=[4097, 33], seed=100 + j)
        sets.append(_sets(clients)[2])
    want = [ops.pairgram_rows_dist(rs, _GRAM_TOL)[0].cpu().numpy()
            for rs in sets]
    for rnd in range(2):
        for j, rs in enumerate(sets):
            got = ops.pairgram_rows_dist_graph(rs, _GRAM_TOL)[0].cpu()
            assert got.numpy().tobytes() == want[j].tobytes(), (rnd, j)
