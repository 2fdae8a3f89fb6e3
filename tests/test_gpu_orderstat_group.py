"""The K-wave order-statistic kernel (csrc/orderstat_group.h): 255 < n <=
512 clients, each column's rows split over K = ceil(n / 64) waves of one
workgroup, read once from HBM.  Against the CPU oracle (median bit-exact,
trimmed mean within tests/trimmed_bounds.py's regression bound) and against the two-pass
streaming kernel on the same inputs (fsagg_orderstat_set_group_max moves
the dispatch)."""
import contextlib

import numpy as np
import pytest
import torch

import oracle as O
from test_gpu_orderstat_pair import columns, trimmed_tol

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def group_max(n):
    from federatedscope_amd import _lib as L
    lib = L.load()
    prev = lib.fsagg_orderstat_set_group_max(int(n))
    try:
        yield
    finally:
        lib.fsagg_orderstat_set_group_max(prev)


@pytest.mark.parametrize('n', [256, 257, 300, 319, 320, 321, 383, 384, 385,
                               448, 449, 500, 511, 512])
def test_group_kernel_vs_oracle_and_stream(n):
    from federatedscope_amd import ops
    P = 64 * 21 + 7
    X = columns(n, P, seed=1000 + n)
    slab = torch.from_numpy(X).cuda()
    rows = ops.RowTable.from_slab(slab)
    base = torch.from_numpy(np.random.default_rng(2).standard_normal(
        P).astype(np.float32)).cuda()
    models = [(1, {'w': X[i]}) for i in range(n)]
    res = {}
    for tag, thr in (('group', 512), ('stream', 255)):
        r = res[tag] = {}
        with group_max(thr):
            out = torch.empty(P, device='cuda')
            ops.coord_median(rows, out)
            r['median'] = out.cpu().numpy()
            ops.coord_median(rows, out, base=base)
            r['median_base'] = out.cpu().numpy()
            for ratio in (0.0, 0.1, 0.2, 0.45):
                k = int(n * ratio)
                ops.trimmed_mean(rows, k, out)
                r[k] = out.cpu().numpy()
    want = O.median_update(models)['w']
    m = res['group']['median']
    assert np.array_equal(m, want)
    keep = np.arange(P) != 7
    assert m[keep].tobytes() == want[keep].tobytes()
    assert m.tobytes() == res['stream']['median'].tobytes()
    assert res['group']['median_base'].tobytes() == \
        res['stream']['median_base'].tobytes()
    for ratio in (0.0, 0.1, 0.2, 0.45):
        k = int(n * ratio)
        want = O.trimmed_mean_update(models, k)['w']
        err = np.abs(res['group'][k].astype(np.float64) - want)
        tol = trimmed_tol(X, k, want, res['group'][k],
                          'group|n%d|k%d' % (n, k))
        assert (err <= tol).all(), (n, k, err.max())


@pytest.mark.parametrize('n', [300, 512])
def test_group_kernel_refinement_and_nonfinite(n):
    from federatedscope_amd import ops
    rng = np.random.default_rng(11 + n)
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
    rows = ops.RowTable.from_slab(torch.from_numpy(X).cuda())
    models = [(1, {'w': X[i]}) for i in range(n)]
    out = torch.empty(P, device='cuda')
    with group_max(512):
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
                              want[fin], g[fin],
                              'group_refine|n%d|k%d' % (n, k))
            assert (err <= tol).all(), (k, err.max())


def test_group_kernel_row_sets():
    """Row-set form (chunk quarters, short chunks) equals the flat form."""
    from collections import OrderedDict

    from federatedscope_amd import ops
    from federatedscope_amd.layout import BucketLayout, ClientStack
    n = 300
    sizes = [1, 1023, 5, 30_001, 3, 257, 64, 65, 191, 192, 193]
    g = torch.Generator(device='cuda').manual_seed(5)
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
    with group_max(512):
        for k in (None, int(n * 0.2)):
            a = torch.full((lay.numel, ), 3.0, device='cuda')
            b = torch.full((lay.numel, ), 3.0, device='cuda')
            if k is None:
                ops.coord_median_rows(rs, a, base=ops.BaseRows.from_bucket(
                    base))
                ops.coord_median(rows, b, base=base)
            else:
                ops.trimmed_mean_rows(rs, k, a)
                ops.trimmed_mean(rows, k, b)
            for key in lay.keys:
                o, m = lay.offsets[key], lay.numels[key]
                assert torch.equal(a[o:o + m], b[o:o + m]), (k, key)
