"""The Krum selection certificate (core/aggregators/_engine.certified_selection)
on the host: when it certifies a selection from D and per-pair bounds B,
every distance matrix within B of D must give that selection (checked by
sampling perturbations at the bounds' corners); zero bounds certify any
selection without ties; bounds wider than the score gaps do not."""
import numpy as np
import pytest
import torch

from federatedscope_amd.core.aggregators._engine import certified_selection
from federatedscope_amd.core.aggregators.krum_aggregator import krum_scores


def _D(n, rng, spread=1.0):
    X = rng.standard_normal((n, 8)) * (1 + spread * rng.random((n, 1)))
    D = np.sqrt(((X[:, None] - X[None]) ** 2).sum(-1)).astype(np.float32)
    np.fill_diagonal(D, np.inf)
    return D


def _sel(D, f, m):
    s = krum_scores(torch.from_numpy(np.asarray(D, np.float32)), f)
    return torch.sort(s)[1].numpy()[:m].tolist()


@pytest.mark.parametrize('seed', range(6))
@pytest.mark.parametrize('ordered', [True, False])
def test_certified_selection_is_stable_under_bounded_perturbation(seed,
                                                                  ordered):
    rng = np.random.default_rng(seed)
    n, f, m = 20, 3, 4
    D = _D(n, rng)
    order = torch.sort(krum_scores(torch.from_numpy(D), f))[1].numpy()
    base = _sel(D, f, m)
    hits = 0
    for scale in (1e-7, 1e-4, 1e-3, 1e-2, 5e-2):
        B = scale * np.where(np.isfinite(D), D, 0.0).astype(np.float64)
        B = np.maximum(B, B.T)
        if not certified_selection(D, B, f, m, order, ordered):
            continue
        hits += 1
        for _ in range(40):
            sgn = rng.choice([-1.0, 1.0], size=(n, n))
            sgn = np.triu(sgn, 1)
            sgn = sgn + sgn.T
            Dp = (D.astype(np.float64) + sgn * B).astype(np.float32)
            np.fill_diagonal(Dp, np.inf)
            got = _sel(Dp, f, m)
            if ordered:
                assert got == base, (scale, got, base)
            else:
                assert sorted(got) == sorted(base), (scale, got, base)
    assert hits >= 1


def test_certificate_zero_bounds_and_ties():
    rng = np.random.default_rng(7)
    n, f = 12, 2
    D = _D(n, rng)
    order = torch.sort(krum_scores(torch.from_numpy(D), f))[1].numpy()
    assert certified_selection(D, np.zeros((n, n)), f, 3, order, True)
    # two identical clients: equal scores, their order is not certifiable
    X = rng.standard_normal((n, 4))
    X[5] = X[2]
    D2 = np.sqrt(((X[:, None] - X[None]) ** 2).sum(-1)).astype(np.float32)
    np.fill_diagonal(D2, np.inf)
    s = krum_scores(torch.from_numpy(D2), f)
    order2 = torch.sort(s)[1].numpy()
    pos = sorted([int(np.nonzero(order2 == 2)[0][0]),
                  int(np.nonzero(order2 == 5)[0][0])])
    B0 = np.zeros((n, n))
    assert not certified_selection(D2, B0, f, pos[1], order2, True)
    # huge bounds certify nothing
    assert not certified_selection(D, np.full((n, n), 1e3), f, 3, order,
                                   False)


def test_certificate_infinite_bound_fails():
    rng = np.random.default_rng(3)
    n, f = 10, 1
    D = _D(n, rng)
    order = torch.sort(krum_scores(torch.from_numpy(D), f))[1].numpy()
    B = np.zeros((n, n))
    B[order[0], order[1]] = B[order[1], order[0]] = np.inf
    assert not certified_selection(D, B, f, 2, order, True)


def _exact_D(X):
    D = np.sqrt(((X[:, None] - X[None]) ** 2).sum(-1))
    np.fill_diagonal(D, np.inf)
    return D


@pytest.mark.parametrize('ordered', [True, False])
def test_refine_selection_recovers_the_exact_selection(ordered):
    """The ambiguous clients' rows replaced by exact ones
    (_engine.refine_selection): when it certifies, the selection is the
    exact distances' one; the rows it asks for are the ambiguous ones."""
    from federatedscope_amd.core.aggregators._engine import (
        ambiguous_clients, refine_selection)
    hits = 0
    for seed in range(30):
        rng = np.random.default_rng(100 + seed)
        n, f = 24, 4
        m = 6 if ordered else n - 2 * f
        X = rng.standard_normal((n, 16))
        De = _exact_D(X)
        eps = 3e-4
        B = eps * np.where(np.isfinite(De), De, 0.0)
        noise = rng.uniform(-1, 1, (n, n)) * B
        noise = np.triu(noise, 1) + np.triu(noise, 1).T
        D = (De + noise).astype(np.float32)
        np.fill_diagonal(D, np.inf)
        order = torch.sort(krum_scores(torch.from_numpy(D), f))[1].numpy()
        amb = ambiguous_clients(D, B, f, m, order, ordered)
        if not amb:
            continue
        asked = []

        def rows(sel):
            asked.append(list(sel))
            return De[sel]
        got = refine_selection(D, B, f, m, ordered, amb, rows, 1e-14, 32)
        assert asked[0] == sorted(amb)
        if got is None:
            continue
        hits += 1
        sc, o, nrows = got
        want = np.argsort(np.sort(De, 1)[:, :n - f - 2].sum(1),
                          kind='stable')
        if ordered:
            assert o[:m].tolist() == want[:m].tolist(), seed
        else:
            assert sorted(o[:m].tolist()) == sorted(want[:m].tolist()), seed
        assert nrows == sum(len(a) for a in asked)
    assert hits >= 3


def test_refine_selection_gives_up_on_ties_and_nonfinite():
    from federatedscope_amd.core.aggregators._engine import (
        ambiguous_clients, refine_selection)
    rng = np.random.default_rng(5)
    n, f = 12, 2
    X = rng.standard_normal((n, 4))
    X[7] = X[3]                       # equal exact scores
    De = _exact_D(X)
    B = 1e-3 * np.where(np.isfinite(De), De, 0.0)
    D = De.astype(np.float32)
    order = torch.sort(krum_scores(torch.from_numpy(D), f))[1].numpy()
    m = n - 1
    amb = ambiguous_clients(D, B, f, m, order, True)
    assert 3 in amb and 7 in amb
    assert refine_selection(D, B, f, m, True, amb, lambda s: De[s], 1e-14,
                            32) is None
    bad = De.copy()
    bad[3, 0] = np.nan
    assert refine_selection(D, B, f, m, True, amb, lambda s: bad[s], 1e-14,
                            32) is None
    # more rows than allowed
    assert refine_selection(D, B, f, m, True, amb, lambda s: De[s], 1e-14,
                            1) is None


def _gram_buffer(D64, Bf, flags=None):
    n = D64.shape[0]
    buf = np.zeros((5, n, n), dtype=np.int32)
    buf[0:2].reshape(-1).view(np.float64)[:] = D64.reshape(-1)
    buf[2] = D64.astype(np.float32).view(np.int32)
    if flags is not None:
        buf[3] = flags
    buf[4] = Bf.astype(np.float32).view(np.int32)
    return buf


@pytest.mark.parametrize('ordered', [True, False])
def test_native_certificate_matches_python(ordered):
    """_fsagg_host.gram_select (csrc/host/krumcert.cpp) against the Python
    restatement: the same ambiguous set and, when certified, the same
    selection."""
    from federatedscope_amd import _lib
    from federatedscope_amd.core.aggregators._engine import ambiguous_clients
    host = _lib.host()
    seen = set()
    for seed in range(40):
        rng = np.random.default_rng(seed)
        n, f = int(rng.integers(6, 60)), int(rng.integers(0, 5))
        m = int(rng.integers(1, n + 1)) if ordered else max(1, n - 2 * f)
        nseg = int(rng.integers(1, 12))
        X = rng.standard_normal((n, 8))
        D64 = np.sqrt(((X[:, None] - X[None]) ** 2).sum(-1))
        np.fill_diagonal(D64, np.inf)
        scale = 10.0 ** rng.uniform(-7, -2)
        Bf = (scale * np.where(np.isfinite(D64), D64, 0.0) *
              rng.random((n, n))).astype(np.float32)
        np.fill_diagonal(Bf, 0)
        got = host.gram_select(_gram_buffer(D64, Bf), nseg, f, m, ordered)
        B64 = np.maximum(Bf, Bf.T).astype(np.float64) + (nseg + 2) * \
            2.0 ** -52 * np.where(np.isfinite(D64), D64, 0.0)
        k = n - f - 2
        if k <= 0:
            assert got is None
            continue
        sc = np.sort(D64, 1)[:, :k].sum(1)
        order = np.argsort(sc, kind='stable')
        want = ambiguous_clients(D64, B64, f, m, order, ordered)
        g_sc, g_order, g_amb = got
        g_sc = np.frombuffer(g_sc, dtype=np.float64)
        g_order = np.frombuffer(g_order, dtype=np.int64).tolist()
        assert np.allclose(g_sc, sc, rtol=1e-14)
        assert g_amb == want, (seed, g_amb, want)
        if not want:
            if ordered:
                assert g_order[:m] == order[:m].tolist()
            else:
                assert sorted(g_order[:m]) == sorted(order[:m].tolist())
        seen.add(bool(want))
    assert seen == {True, False}
    # a flagged pair: the caller's repair path
    D64 = np.ones((4, 4))
    np.fill_diagonal(D64, np.inf)
    fl = np.zeros((4, 4), dtype=np.int32)
    fl[1, 2] = 1
    assert host.gram_select(_gram_buffer(D64, np.zeros((4, 4)), fl), 1, 0,
                            1, True) is None
