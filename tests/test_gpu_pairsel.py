"""Krum distances of a few selected clients to every client in fp64
(fsagg_pairsel_rows_segsq_f64 + fsagg_pairsel_finish_f64), and the
selection refinement that uses them (_engine.refine_selection): when the
Gram path's bounds leave a Krum / Bulyan selection ambiguous, only the
ambiguous clients' rows are recomputed.

* the kernel against fp64 numpy on the same rows: n = 2 … 256 (1–4 waves
  per client set), 1 … 32 selected rows (every accumulator-array size),
  keys of 0 … 300k elements, keyed and stacked row sets and rows that are
  not 16-B aligned (the per-element load path);
* the engine on "twin" clients — each client's mirror image −x, nudged so
  the twins' Krum scores differ by ~1e-8 relative, far inside the Gram
  path's bounds: the multi-Krum order and the Bulyan set are the fp64
  distances' selection, decided from the recomputed rows alone (path
  'mfma + exact rows …', no full recomputation)."""
from collections import OrderedDict
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from test_gpu_pairgram import SIZES, _as_slab, _clients, _DictModel, _sets

pytestmark = pytest.mark.gpu


def _rows_fp64(clients, lay, sel):
    """[nseg][len(sel)][n] fp64 per-key squared distances."""
    out = np.zeros((len(lay.keys), len(sel), len(clients)))
    for s, k in enumerate(lay.keys):
        X = np.stack([c[k].double().cpu().numpy().ravel() for c in clients])
        for i, a in enumerate(sel):
            out[s, i] = ((X - X[a]) ** 2).sum(axis=1)
    return out


def _check_rows(rs, clients, lay, sel):
    from federatedscope_amd import ops
    sel_t = torch.tensor(sel, dtype=torch.int32, device='cuda')
    sq = ops.pairsel_rows_segsq(rs, sel_t)
    D = ops.pairsel_finish(sq, sel_t).cpu().numpy()
    sq = sq.cpu().numpy()
    want = _rows_fp64(clients, lay, sel)
    big = max(lay.numels.values())
    rel = (big + 64) * 2.0 ** -53
    assert np.all(np.abs(sq - want) <= rel * want + 1e-300), \
        float(np.max(np.abs(sq - want) / np.maximum(want, 1e-300)))
    Dw = np.sqrt(want).sum(0)
    for i, a in enumerate(sel):
        assert D[i, a] == np.inf
        Dw[i, a] = np.inf
    fin = np.isfinite(Dw)
    assert np.all(np.abs(D[fin] - Dw[fin]) <= 1e-12 * Dw[fin])


@pytest.mark.parametrize('n,sel', [
    (2, [1]), (5, [0, 4, 2]), (50, [3, 7, 11, 19, 49]),
    (64, list(range(0, 64, 4))), (65, list(range(0, 65, 2))[:17]),
    (129, [128, 0, 64, 65, 1, 2, 3, 4, 5]),
    (200, list(range(0, 200, 7))[:28]), (256, list(range(255, -1, -8)))])
def test_pairsel_vs_fp64(n, sel):
    sizes = SIZES if n <= 64 else [1, 0, 1023, 5, 30_001, 3, 7, 4099, 33]
    clients = _clients(n, sizes=sizes, seed=n)
    lay, _, keyed, stacked = _sets(clients)
    _check_rows(keyed, clients, lay, sel)
    _check_rows(stacked, clients, lay, sel)


def test_pairsel_unaligned_rows():
    from federatedscope_amd import ops
    n = 40
    clients = _clients(n, sizes=[1023, 70_001, 5], seed=3)
    keys = list(clients[0].keys())
    slab = torch.zeros((n, 80_000), device='cuda')
    views = []
    for i, c in enumerate(clients):
        d, o = OrderedDict(), 1 + i % 3           # 4-B offsets: unaligned
        for k in keys:
            m = c[k].numel()
            d[k] = slab[i, o:o + m]
            d[k].copy_(c[k])
            o += m + 1
        views.append(d)
    lay, _, keyed, _ = _sets(views)
    _check_rows(keyed, views, lay, [0, 5, 39])
    with pytest.raises(ValueError):
        ops.pairsel_rows_segsq(keyed, torch.zeros(33, dtype=torch.int32,
                                                  device='cuda'))


TWIN_SIZES = [100_003, 4097, 33, 65_536, 7]


def _twins(h=25, delta=1e-4, seed=17):
    """h clients, their mirror images (nudged by delta·noise) and one far
    client: the twins' Krum scores tie up to O(delta)."""
    g = torch.Generator(device='cuda').manual_seed(seed)
    base = [OrderedDict(('k%d' % j, torch.randn(sz, device='cuda',
                                                generator=g))
                        for j, sz in enumerate(TWIN_SIZES))
            for _ in range(h)]
    out = []
    for c in base:
        out.append(c)
        out.append(OrderedDict(
            (k, -v + delta * torch.randn(v.shape, device='cuda', generator=g))
            for k, v in c.items()))
    out.append(OrderedDict(
        (k, 4.0 * torch.randn(v.shape, device='cuda', generator=g))
        for k, v in base[0].items()))
    return out


def _cfg(f, m):
    return SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=1000, sample_client_rate=1.0),
        aggregator=SimpleNamespace(
            byzantine_node_num=f,
            BFT_args=SimpleNamespace(krum_agg_num=m)))


def _exact_scores(clients, f):
    from federatedscope_amd.layout import BucketLayout
    lay = BucketLayout(OrderedDict((k, v.cpu()) for k, v in
                                   clients[0].items()))
    n = len(clients)
    D = np.sqrt(_rows_fp64(clients, lay, list(range(n)))).sum(0)
    np.fill_diagonal(D, np.inf)
    return np.sort(D, 1)[:, :n - f - 2].sum(1)


@pytest.mark.parametrize('rule', ['multi_krum', 'bulyan'])
def test_refined_selection_on_twins(rule):
    from federatedscope_amd.core.aggregators import (BulyanAggregator,
                                                     KrumAggregator)
    clients = _twins()
    n, f = len(clients), 10
    sc = _exact_scores(clients, f)
    want = np.argsort(sc, kind='stable')
    init = OrderedDict((k, torch.zeros_like(v)) for k, v in
                       clients[0].items())
    feed = {'client_feedback': [(1, c) for c in _as_slab(clients)],
            'recover_fun': None}
    if rule == 'multi_krum':
        m = 5
        agg = KrumAggregator(model=_DictModel(init), device='cuda',
                             config=_cfg(f, m))
        agg.aggregate(feed)
        assert agg.last_selection == want[:m].tolist()
    else:
        m = n - 2 * f                       # 31: the cut splits a twin pair
        agg = BulyanAggregator(model=_DictModel(init), device='cuda',
                               config=_cfg(f, 1))
        agg.aggregate(feed)
        assert sorted(agg.last_selection) == sorted(want[:m].tolist())
        # the twins at the cut really are closer than the Gram bounds
        gap = (sc[want[m]] - sc[want[m - 1]]) / sc[want[m]]
        assert gap < 1e-6, gap
    assert agg.last_pairdist_path.startswith('mfma + exact rows'), \
        agg.last_pairdist_path
