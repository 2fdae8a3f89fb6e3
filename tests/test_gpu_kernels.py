"""Kernel-level parity on the GPU against the CPU oracle, across the launch
shapes each kernel picks (every V of the weighted sum, ragged tails, the
register-sort / register-radix / generic order-statistic kernels), plus the
edge cases the reference's rules have (n = 1, ties, ±inf, NaN)."""
import numpy as np
import pytest
import torch

import oracle as O
import trimmed_bounds as TB

pytestmark = pytest.mark.gpu


def _slab(n, P, seed):
    from federatedscope_amd import ops
    ld = ops.round_up(max(P, 1), 64)
    slab = torch.empty((n, ld), device='cuda')
    ops.fill_uniform(slab, P, seed=seed)
    return slab


def _host_uniform(n, P, seed, off=0):
    """The on-device generator restated on the host (uint64 wrap-around)."""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)
    c = np.arange(n, dtype=np.uint64)[:, None]
    j = np.arange(P, dtype=np.uint64)[None, :] + np.uint64(off)
    with np.errstate(over='ignore'):
        z = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)) & M
        z = z ^ (c << np.uint64(40)) ^ j
        z ^= z >> np.uint64(30)
        z = z * np.uint64(0xBF58476D1CE4E5B9)
        z ^= z >> np.uint64(27)
        z = z * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return ((z >> np.uint64(40)).astype(np.float32) * np.float32(2**-23) -
            np.float32(1.0))


def test_fill_uniform_matches_host_generator():
    slab = _slab(3, 1000, seed=77)
    want = _host_uniform(3, 1000, 77)
    assert slab[:, :1000].cpu().numpy().tobytes() == want.tobytes()


@pytest.mark.parametrize('P', [1, 3, 4, 5, 1023, 4097, 1_000_003, 5_000_000,
                               9_000_001, 17_000_002, 25_000_003])
def test_weighted_sum_all_shapes(P):
    from federatedscope_amd import ops
    n = 5 if P > 1_000_000 else 17
    slab = _slab(n, P, seed=P)
    sizes = [(i * 37) % 101 + 1 for i in range(n)]
    w = O.fedavg_weights(sizes)
    out = torch.empty(ops.round_up(P, 4), device='cuda')[:P]
    ops.weighted_sum(ops.RowTable.from_slab(slab, numel=P), w, out)
    X = slab[:, :P].cpu().numpy()
    want = O.para_weighted_avg([(s, {'w': X[i]}) for i, s in
                                enumerate(sizes)])['w']
    assert out.cpu().numpy().tobytes() == want.tobytes()


def test_weighted_sum_prescale_and_base():
    from federatedscope_amd import ops
    n, P = 6, 100_001
    slab = _slab(n, P, seed=3)
    base = torch.randn(P + 3, device='cuda')[:P].contiguous()
    w = O.fedavg_weights([3, 1, 4, 1, 5, 9])
    pre = [1.0, 0.5, 1.0, 0.123456789, 2.0, 1.0]
    out = torch.empty(P, device='cuda')
    ops.weighted_sum(ops.RowTable.from_slab(slab, numel=P), w, out,
                     prescale=pre, base=base)
    X = slab[:, :P].cpu().numpy()
    acc = None
    for i in range(n):
        t = (X[i] * np.float32(pre[i])) * np.float32(w[i])
        acc = t if acc is None else acc + t
    want = base.cpu().numpy() + acc
    assert out.cpu().numpy().tobytes() == want.tobytes()


def test_weighted_sum_row_order_is_reduction_order():
    """Reordering the row table reorders the fp32 sum (as the reference's
    client list order does) — the kernel must follow the table."""
    from federatedscope_amd import ops
    n, P = 40, 65536
    slab = _slab(n, P, seed=8) * 1000
    w = [1.0 / 3.0] * n
    a = torch.empty(P, device='cuda')
    b = torch.empty(P, device='cuda')
    ops.weighted_sum(ops.RowTable.from_slab(slab, numel=P), w, a)
    perm = list(reversed(range(n)))
    ops.weighted_sum(ops.RowTable.from_slab(slab, rows=perm, numel=P), w, b)
    X = slab[:, :P].cpu().numpy()
    wa = O.para_weighted_avg([(1, {'w': X[i]}) for i in range(n)],
                             weights=w)['w']
    wb = O.para_weighted_avg([(1, {'w': X[i]}) for i in perm],
                             weights=w)['w']
    assert a.cpu().numpy().tobytes() == wa.tobytes()
    assert b.cpu().numpy().tobytes() == wb.tobytes()


@pytest.mark.parametrize('n', [1, 2, 3, 4, 7, 8, 31, 32, 33, 40, 41, 48, 50,
                               56, 57, 64, 65, 72, 73, 100, 127, 200, 233,
                               250, 255, 256, 257, 300, 511, 1000, 2049])
def test_median_trimmed_all_kernels(n):
    """Every order-statistic kernel (register network n <= 32 and
    56 < n <= 64, register select 32 < n <= 56 and 64 < n <= 255, streaming
    select n > 255) against the oracle on
    ties, signed zeros and columns spanning > 16 octaves (the refinement
    rounds)."""
    from federatedscope_amd import ops
    P = 3001
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, P)).astype(np.float32)
    X[:, 5] = 1.5                   # all tied
    X[:, 6] = np.float32(rng.integers(0, 3, n))  # heavy ties
    X[:, 7] = -0.0
    X[: max(1, n // 10), 8] *= 1e30
    # large values only past the first 64 rows (the streaming kernel's
    # base sample) and a column whose magnitudes grow down the rows
    X[n - max(1, n // 5):, 9] *= 1e6
    X[:, 10] = np.float32(np.linspace(-1, 1, n) * np.logspace(0, 20, n))
    slab = torch.from_numpy(X).cuda()
    rows = ops.RowTable.from_slab(slab)
    out = torch.empty(P, device='cuda')
    ops.coord_median(rows, out)
    models = [(1, {'w': X[i]}) for i in range(n)]
    want = O.median_update(models)['w']
    got = out.cpu().numpy()
    # -0/+0 ties may pick either zero; compare values, and bits elsewhere
    assert np.array_equal(got, want)
    assert got[np.arange(P) != 7].tobytes() == \
        want[np.arange(P) != 7].tobytes(), n
    for ratio in (0.0, 0.1, 0.2, 0.45):
        k = int(n * ratio)
        if 2 * k >= n:
            continue
        ops.trimmed_mean(rows, k, out)
        want = O.trimmed_mean_update(models, k)['w']
        eps = np.finfo(np.float32).eps
        g = out.cpu().numpy()
        T = np.stack([m[1]['w'] for m in models])
        TB.check_vs_oracle('kernels|n%d|k%d' % (n, k), g, want, T, n - 2 * k)


def test_orderstat_nonfinite_columns():
    from federatedscope_amd import ops
    n, P = 9, 8
    X = np.ones((n, P), np.float32)
    X[0, 0] = np.nan
    X[0, 1] = np.inf
    X[0, 2] = -np.inf
    X[1, 3] = np.inf
    X[2, 3] = -np.inf
    slab = torch.from_numpy(X).cuda()
    rows = ops.RowTable.from_slab(slab)
    out = torch.empty(P, device='cuda')
    ops.coord_median(rows, out)
    m = out.cpu().numpy()
    assert np.isnan(m[0]) and m[1] == 1.0 and m[2] == 1.0 and m[3] == 1.0
    ops.trimmed_mean(rows, 2, out)
    t = out.cpu().numpy()
    # the reference's Σall − Σtop − Σbottom: any ±inf with k >= 1 → NaN
    assert np.isnan(t[:4]).all() and (t[4:] == 1.0).all()
    ops.trimmed_mean(rows, 0, out)
    t = out.cpu().numpy()
    assert np.isnan(t[0]) and t[1] == np.inf and t[2] == -np.inf and \
        np.isnan(t[3])


@pytest.mark.parametrize('n', [2, 3, 9, 21, 25, 33, 45, 50, 64, 100, 200])
def test_pairdist_vs_fp64(n):
    from federatedscope_amd import ops
    P = 20_011
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, P)).astype(np.float32)
    offs = [0, 1, 17, 4000, 4001, P]
    slab = torch.from_numpy(X).cuda()
    D = ops.pairdist(ops.RowTable.from_slab(slab), offs).cpu().numpy()
    paras = [{'k%d' % s: X[i, offs[s]:offs[s + 1]] for s in range(5)}
             for i in range(n)]
    Dref = O.krum_distance_matrix(paras)
    off = ~np.eye(n, dtype=bool)
    np.testing.assert_allclose(D[off], Dref[off], rtol=2e-6)
    assert np.isinf(np.diag(D)).all()
    assert np.array_equal(D, D.T)


def test_row_sqnorm_vs_fp64():
    from federatedscope_amd import ops
    n, P = 7, 1_000_001
    slab = _slab(n, P, seed=4)
    sq = ops.row_sqnorm(ops.RowTable.from_slab(slab, numel=P)).cpu().numpy()
    X = slab[:, :P].cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(sq, (X * X).sum(1), rtol=1e-12)


@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16, torch.float64,
                                torch.int64])
def test_typed_weighted_sum(dt):
    from federatedscope_amd import ops
    n, P = 13, 4099
    g = torch.Generator().manual_seed(1)
    if dt == torch.int64:
        xs = [torch.randint(-10**6, 10**6, (P, ), generator=g)
              for _ in range(n)]
    else:
        xs = [torch.randn(P, generator=g).to(dt) for _ in range(n)]
    w = O.fedavg_weights([i + 1 for i in range(n)])
    out = torch.empty(P, dtype=ops.typed_out_dtype(dt), device='cuda')
    ops.weighted_sum_typed([x.cuda() for x in xs], w, out)
    # the reference's own semantics, via the oracle
    def np_of(x):
        if dt == torch.bfloat16:
            return O.BF16(x.view(torch.int16).numpy().view(np.uint16))
        return x.numpy()
    want = O.para_weighted_avg([(1, {'w': np_of(x)}) for x in xs],
                               weights=w)['w']
    got = out.cpu()
    if dt == torch.bfloat16:
        assert np.array_equal(got.view(torch.int16).numpy().view(np.uint16),
                              want.bits)
    else:
        assert got.numpy().tobytes() == np.asarray(want).tobytes()


@pytest.mark.parametrize('n', [9, 65, 100, 200, 255, 300, 1000])
def test_orderstat_nonfinite_columns_all_kernels(n):
    """±inf / NaN columns through every order-statistic kernel (the
    register network, the select kernels and the streaming n > 255 path)."""
    from federatedscope_amd import ops
    P = 8
    X = np.ones((n, P), np.float32)
    X[0, 0] = np.nan
    X[0, 1] = np.inf
    X[0, 2] = -np.inf
    X[1, 3] = np.inf
    X[2, 3] = -np.inf
    X[:, 4] = np.float32(np.arange(n) % 5)
    X[3:, 5] = np.inf                    # mostly +inf
    slab = torch.from_numpy(X).cuda()
    rows = ops.RowTable.from_slab(slab)
    out = torch.empty(P, device='cuda')
    ops.coord_median(rows, out)
    models = [(1, {'w': X[i]}) for i in range(n)]
    want = O.median_update(models)['w']
    assert np.array_equal(out.cpu().numpy(), want, equal_nan=True)
    for k in (0, 1, n // 5):
        if 2 * k >= n:
            continue
        ops.trimmed_mean(rows, k, out)
        want = O.trimmed_mean_update(models, k)['w']
        got = out.cpu().numpy()
        assert np.array_equal(np.isnan(got), np.isnan(want)), (k, got, want)
        fin = np.isfinite(want)
        assert np.array_equal(got[~fin & ~np.isnan(want)],
                              want[~fin & ~np.isnan(want)])
        np.testing.assert_allclose(got[fin], want[fin], rtol=1e-6)


@pytest.mark.parametrize('n', [100, 200, 255])
def test_orderstat_refinement_stress(n):
    """Columns built to drive the select kernel through every refinement
    shape: a heavy cluster within a few ulps (bins refined down to lvl < 7),
    two far clusters (dual refinement), a tight cluster next to a single
    outlier, and wide dynamic ranges — median bit-exact, trimmed mean within
    the summation tolerance."""
    from federatedscope_amd import ops
    rng = np.random.default_rng(100 + n)
    cols = []
    one = np.float32(1.0)
    ulps = np.nextafter(one, np.float32(2)) - one
    c = np.full(n, one, np.float32) + ulps * rng.integers(0, 4, n)
    c[: n // 4] = 3.0
    c[n // 4] = 2.0
    cols.append(c)                                    # ulp cluster
    c = np.where(rng.random(n) < 0.5,
                 -5.0 + 1e-6 * rng.standard_normal(n),
                 7.0 + 1e-6 * rng.standard_normal(n)).astype(np.float32)
    cols.append(c)                                    # two tight clusters
    c = (1e-3 * rng.standard_normal(n)).astype(np.float32)
    c[0] = 1e30
    cols.append(c)                                    # one huge outlier
    c = (rng.standard_normal(n) * 10.0 ** rng.integers(-20, 20, n)).astype(
        np.float32)
    cols.append(c)                                    # wide exponents
    c = np.float32(rng.integers(-2, 3, n)) + np.float32(1e-7) * \
        np.float32(rng.integers(0, 2, n))
    cols.append(c.astype(np.float32))                 # ties + near ties
    c = rng.standard_normal(n).astype(np.float32)
    c[rng.random(n) < 0.1] *= 100.0
    cols.append(c)                                    # C5-like
    X = np.stack(cols, 1).astype(np.float32)
    X = np.repeat(X, 70, axis=1)                      # > one wave of columns
    for j in range(X.shape[1]):
        X[:, j] = X[rng.permutation(n), j]
    P = X.shape[1]
    slab = torch.from_numpy(np.ascontiguousarray(X)).cuda()
    rows = ops.RowTable.from_slab(slab)
    out = torch.empty(P, device='cuda')
    models = [(1, {'w': X[i]}) for i in range(n)]
    ops.coord_median(rows, out)
    assert out.cpu().numpy().tobytes() == \
        O.median_update(models)['w'].tobytes()
    eps = np.finfo(np.float32).eps
    for k in (1, n // 5, n // 2 - 1):
        ops.trimmed_mean(rows, k, out)
        want = O.trimmed_mean_update(models, k)['w']
        g = out.cpu().numpy()
        T = np.stack([m[1]['w'] for m in models])
        TB.check_vs_oracle('stream|n%d|k%d' % (n, k), g, want, T, n - 2 * k)


@pytest.mark.parametrize('n', [12, 50, 130, 255, 256, 300])
def test_pairdist_aligned_rows_stage_plans(n):
    """16-B aligned rows (the production ClientStack layout) take the
    register-prefetched full-stage path; the client counts cover every stage
    plan shape (k-slices > 1 with lcm(4, ks) stages, one k-slice, stages
    capped by the LDS or by the prefetch registers)."""
    from federatedscope_amd import ops
    P = 6007
    ld = ops.round_up(P, 64)
    rng = np.random.default_rng(1000 + n)
    X = np.zeros((n, ld), np.float32)
    X[:, :P] = rng.standard_normal((n, P)).astype(np.float32)
    offs = [0, 3, 2500, 2501, P]
    slab = torch.from_numpy(X).cuda()
    rows = ops.RowTable.from_slab(slab, numel=P)
    assert rows.aligned16
    D = ops.pairdist(rows, offs).cpu().numpy()
    X64 = X[:, :P].astype(np.float64)
    Dref = np.zeros((n, n), np.float32)
    for s in range(len(offs) - 1):
        blk = X64[:, offs[s]:offs[s + 1]]
        for a in range(n):
            Dref[a] += np.sqrt(((blk - blk[a]) ** 2).sum(1)).astype(
                np.float32)
    off = ~np.eye(n, dtype=bool)
    np.testing.assert_allclose(D[off], Dref[off], rtol=2e-6)
    assert np.isinf(np.diag(D)).all()
