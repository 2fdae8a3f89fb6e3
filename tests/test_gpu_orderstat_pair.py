"""The two-wave order-statistic kernel (csrc/orderstat_pair.h): each
column's rows split over two waves of one workgroup, a shared histogram and
list in LDS.  It serves 64 < n <= 255 from fsagg_orderstat_set_pair_min()'s
threshold up (the default routes n >= 129 to it); here the threshold is
moved so that every register-array size is exercised, against the CPU
oracle (median bit-exact; trimmed mean within the bound its fp32 group sums
carry) and against the one-wave kernel on the same inputs."""
import contextlib

import numpy as np
import pytest
import torch

import oracle as O
import trimmed_bounds as TB

pytestmark = pytest.mark.gpu

EPS = float(np.finfo(np.float32).eps)


@contextlib.contextmanager
def pair_min(n):
    from federatedscope_amd import _lib as L
    lib = L.load()
    prev = lib.fsagg_orderstat_set_pair_min(int(n))
    try:
        yield
    finally:
        lib.fsagg_orderstat_set_pair_min(prev)


def trimmed_tol(X, k, want, got=None, tag='kernel'):
    """|ours − oracle| <= the regression bound of tests/trimmed_bounds.py
    (ORACLE_UNITS·ε·Σ|x|/(n − 2k) + 4ε|want|); with ``got`` the measured
    error is logged ($FSAGG_ERR_LOG)."""
    u = TB.units(X, X.shape[0] - 2 * k)
    slack = 4 * EPS * np.abs(want)
    if got is not None:
        TB.log(tag, np.abs(np.asarray(got, np.float64) - want), u, slack)
    return TB.ORACLE_UNITS * u + slack


def columns(n, P, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, P)).astype(np.float32)
    X[:, 5] = 1.5                                   # all tied
    X[:, 6] = np.float32(rng.integers(0, 3, n))     # heavy ties
    X[:, 7] = -0.0
    X[: max(1, n // 10), 8] *= 1e30                 # > 16 octaves: refine
    X[n - max(1, n // 5):, 9] *= 1e6
    X[:, 10] = np.float32(np.linspace(-1, 1, n) * np.logspace(0, 20, n))
    X[:, 11] = np.float32(1e-40)                    # denormals
    X[rng.random((n, P)) < 0.02] *= 100.0           # C5-like outliers
    return X


@pytest.mark.parametrize('n', [65, 71, 72, 73, 100, 127, 128, 129, 136, 199,
                               200, 201, 233, 250, 254, 255])
def test_pair_kernel_vs_oracle_and_one_wave(n):
    from federatedscope_amd import ops
    P = 64 * 37 + 13                  # a ragged last block
    X = columns(n, P, seed=n)
    slab = torch.from_numpy(X).cuda()
    rows = ops.RowTable.from_slab(slab)
    base = torch.from_numpy(np.random.default_rng(1).standard_normal(
        P).astype(np.float32)).cuda()
    models = [(1, {'w': X[i]}) for i in range(n)]
    got, one = {}, {}
    for tag, thr in (('pair', 65), ('one', 256)):
        res = got if tag == 'pair' else one
        with pair_min(thr):
            out = torch.empty(P, device='cuda')
            ops.coord_median(rows, out)
            res['median'] = out.cpu().numpy()
            ops.coord_median(rows, out, base=base)
            res['median_base'] = out.cpu().numpy()
            for ratio in (0.0, 0.1, 0.2, 0.45):
                k = int(n * ratio)
                ops.trimmed_mean(rows, k, out)
                res[k] = out.cpu().numpy()
    want = O.median_update(models)['w']
    m = got['median']
    assert np.array_equal(m, want)
    keep = np.arange(P) != 7          # -0/+0 ties may pick either zero
    assert m[keep].tobytes() == want[keep].tobytes()
    assert m.tobytes() == one['median'].tobytes()
    assert got['median_base'].tobytes() == one['median_base'].tobytes()
    for ratio in (0.0, 0.1, 0.2, 0.45):
        k = int(n * ratio)
        want = O.trimmed_mean_update(models, k)['w']
        err = np.abs(got[k].astype(np.float64) - want)
        tol = trimmed_tol(X, k, want, got[k], 'pair|n%d|k%d' % (n, k))
        assert (err <= tol).all(), (n, k, err.max())


@pytest.mark.parametrize('n', [130, 200, 255])
def test_pair_kernel_refinement_and_nonfinite(n):
    """The refinement rounds (both waves add into the shared refine
    histogram, the same round count in both) and non-finite columns."""
    from federatedscope_amd import ops
    rng = np.random.default_rng(7 + n)
    one = np.float32(1.0)
    ulps = np.nextafter(one, np.float32(2)) - one
    cols = []
    c = np.full(n, one, np.float32) + ulps * rng.integers(0, 4, n)
    c[: n // 4] = 3.0
    c[n // 4] = 2.0
    cols.append(c)
    cols.append(np.where(rng.random(n) < 0.5,
                         -5.0 + 1e-6 * rng.standard_normal(n),
                         7.0 + 1e-6 * rng.standard_normal(n)))
    c = 1e-3 * rng.standard_normal(n)
    c[0] = 1e30
    cols.append(c)
    cols.append(rng.standard_normal(n) * 10.0 ** rng.integers(-20, 20, n))
    X = np.stack(cols, 1).astype(np.float32)
    X = np.repeat(X, 40, axis=1)
    for j in range(X.shape[1]):
        X[:, j] = X[rng.permutation(n), j]
    nf = np.ones((n, 6), np.float32)
    nf[0, 0] = np.nan
    nf[0, 1] = np.inf
    nf[0, 2] = -np.inf
    nf[1, 3] = np.inf
    nf[2, 3] = -np.inf
    nf[3:, 5] = np.inf
    X = np.ascontiguousarray(np.concatenate([X, nf], 1))
    P = X.shape[1]
    slab = torch.from_numpy(X).cuda()
    rows = ops.RowTable.from_slab(slab)
    models = [(1, {'w': X[i]}) for i in range(n)]
    out = torch.empty(P, device='cuda')
    with pair_min(65):
        ops.coord_median(rows, out)
        assert np.array_equal(out.cpu().numpy(), O.median_update(models)['w'],
                              equal_nan=True)
        for k in (0, 1, n // 5, n // 2 - 1):
            ops.trimmed_mean(rows, k, out)
            want = O.trimmed_mean_update(models, k)['w']
            g = out.cpu().numpy()
            assert np.array_equal(np.isnan(g), np.isnan(want)), k
            fin = np.isfinite(want)
            assert np.array_equal(g[~fin & ~np.isnan(want)],
                                  want[~fin & ~np.isnan(want)])
            err = np.abs(g[fin].astype(np.float64) - want[fin])
            tol = trimmed_tol(np.where(np.isfinite(X), X, 0)[:, fin], k,
                              want[fin], g[fin], 'pair_refine|n%d|k%d' % (n, k))
            assert (err <= tol).all(), (k, err.max())


@pytest.mark.parametrize('n', [100, 200])
def test_pair_kernel_row_sets(n):
    """Row-set form: a chunk's four 64-coordinate quarters, short chunks
    (missing quarters) and keys of 1..257 coordinates — identical to the
    flat form over the same rows."""
    from collections import OrderedDict

    from federatedscope_amd import ops
    from federatedscope_amd.layout import BucketLayout, ClientStack
    sizes = [1, 1023, 5, 70_001, 3, 257, 64, 65, 191, 192, 193]
    g = torch.Generator(device='cuda').manual_seed(n)
    clients = [OrderedDict(('k%d' % j, torch.randn(sz, device='cuda',
                                                   generator=g))
                           for j, sz in enumerate(sizes)) for _ in range(n)]
    lay = BucketLayout(OrderedDict((k, v.cpu()) for k, v in
                                   clients[0].items()))
    st = ClientStack(lay, n, 'cuda')
    st.slab.zero_()
    st.load_many(clients)
    ptrs = np.array([[c[k].data_ptr() for k in lay.keys] for c in clients],
                    dtype=np.int64)
    rs = ops.RowSet.from_pointers(lay, ptrs, 'cuda', keepalive=clients)
    rows = ops.RowTable.from_slab(st.slab, numel=lay.numel)
    base = torch.randn(lay.numel, device='cuda')
    k = int(n * 0.2)
    with pair_min(65):
        a = torch.full((lay.numel, ), 3.0, device='cuda')
        b = torch.full((lay.numel, ), 3.0, device='cuda')
        ops.coord_median_rows(rs, a, base=ops.BaseRows.from_bucket(base))
        ops.coord_median(rows, b, base=base)
        for key in lay.keys:
            o, m = lay.offsets[key], lay.numels[key]
            assert torch.equal(a[o:o + m], b[o:o + m]), key
        ops.trimmed_mean_rows(rs, k, a)
        ops.trimmed_mean(rows, k, b)
        for key in lay.keys:
            o, m = lay.offsets[key], lay.numels[key]
            assert torch.equal(a[o:o + m], b[o:o + m]), key
