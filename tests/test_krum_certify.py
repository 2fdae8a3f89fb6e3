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
