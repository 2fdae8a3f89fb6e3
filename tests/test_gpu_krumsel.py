"""Krum's certified selection on the device (fsagg_krum_select_f32,
csrc/krumsel.hip) against the native host certificate it restates
(_fsagg_host.gram_select, csrc/host/krumcert.cpp, itself checked against
the Python restatement in tests/test_krum_certify.py), and the multi-Krum
drop-in that uses it against the host route, bit for bit.

Finish buffers are synthetic (int32 [5][n][n]: D64, D, flags, B): well
separated scores (certified), near-ties (ambiguous), flagged pairs and
k = n − f − 2 <= 0 (no certificate); ordered and unordered, m >= n."""
from collections import OrderedDict
from types import SimpleNamespace

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _buf(n, seed, family):
    """A finish buffer as ops._gram_buf lays it out (host int32)."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, 6))
    if family == 'separated':
        x *= np.linspace(1.0, 3.0, n)[:, None]     # distinct row scales
    elif family == 'ties':
        x = np.repeat(x[:1], n, 0) + 1e-13 * rng.standard_normal((n, 6))
    D64 = np.sqrt(((x[:, None, :] - x[None, :, :]) ** 2).sum(-1))
    np.fill_diagonal(D64, np.inf)
    B = np.abs(rng.standard_normal((n, n))) * 1e-7 * np.where(
        np.isfinite(D64), D64, 0.0)
    np.fill_diagonal(B, 0.0)
    flags = np.zeros((n, n), dtype=np.uint32)
    if family == 'flagged':
        flags[0, min(1, n - 1)] = 1
    buf = np.zeros((5, n, n), dtype=np.int32)
    buf[0:2] = np.frombuffer(D64.astype(np.float64).tobytes(),
                             dtype=np.int32).reshape(2, n, n)
    buf[2] = D64.astype(np.float32).view(np.int32)
    buf[3] = flags.view(np.int32)
    buf[4] = B.astype(np.float32).view(np.int32)
    return buf


@pytest.mark.parametrize('n', [2, 5, 17, 50, 64, 129, 256])
@pytest.mark.parametrize('family', ['separated', 'random', 'ties',
                                    'flagged'])
def test_device_select_matches_host_certificate(n, family):
    from federatedscope_amd import _lib as L
    from federatedscope_amd import ops
    host = L.host()
    buf = _buf(n, 7 * n + len(family), family)
    dbuf = torch.from_numpy(buf).cuda()
    nseg = 3
    tab = torch.arange(nseg * n, dtype=torch.int64, device='cuda').view(
        nseg, n) * 16 + 4096
    rng = np.random.default_rng(n)
    sizes = [float(s) for s in rng.integers(1, 1000, n)]
    for f in sorted({0, 1, n // 5, max(n - 2, 0)}):
        for m in sorted({1, 3, n - 1, n, n + 2} - {0}):
            for ordered in (True, False):
                want = host.gram_select(buf, nseg, f, m, ordered)
                sel, sub_tab, sub_w, _ = ops.krum_select(
                    dbuf, nseg, f, m, ordered, sizes, False, tab, n, nseg)
                got = sel.cpu().numpy()
                if want is None:
                    assert got[1] == 0 and got[0] == 0, (f, m)
                    continue
                sc, order, amb = want
                order = np.frombuffer(order, dtype=np.int64)
                assert got[1] == 1
                assert bool(got[0]) == (not amb), (f, m, ordered, amb)
                if amb:
                    continue
                msel = min(m, n)
                o = got[2:2 + n]
                if ordered:
                    assert list(o[:msel]) == list(order[:msel])
                else:
                    assert set(o[:msel]) == set(order[:msel])
                # the average's operands: the chosen clients' table rows and
                # fedavg weights (size / total in fp64, then fp32)
                st = sub_tab.cpu().numpy()
                tb = tab.cpu().numpy()
                assert np.array_equal(st, tb[:, o[:msel]])
                tot = 0.0
                for i in o[:msel]:
                    tot += sizes[i]
                w = np.array([sizes[i] / tot for i in o[:msel]],
                             dtype=np.float32)
                assert np.array_equal(sub_w.cpu().numpy(), w)


def _cfg(f, agg, ignore_weight=False):
    bft = SimpleNamespace(krum_agg_num=agg)
    return SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=ignore_weight, use_ss=False,
                                 client_num=1000),
        aggregator=SimpleNamespace(byzantine_node_num=f, BFT_args=bft))


class _Model(torch.nn.Module):
    def __init__(self, sd):
        super().__init__()
        self.sd = sd

    def state_dict(self, *a, **kw):
        return self.sd


KEYS = [('conv.weight', (32, 1, 5, 5)), ('conv.bias', (32, )),
        ('fc.weight', (61, 333)), ('fc.bias', (61, )), ('out', (4099, ))]


@pytest.mark.parametrize('n,f,agg', [(12, 2, 1), (50, 10, 5), (64, 12, 30)])
@pytest.mark.parametrize('where', ['device', 'host'])
@pytest.mark.parametrize('ignore_weight', [False, True])
def test_krum_device_selection_matches_host_route(n, f, agg, where,
                                                  ignore_weight):
    """KrumAggregator.aggregate through the device selection equals the
    host route (its certificate on the finish buffer's host copy, the subset
    row set, fedavg weights on the host) bit for bit, with the same
    selection — on device dicts (keyed rows) and host dicts (stack rows);
    Byzantine clients far from the rest are never chosen."""
    from federatedscope_amd.core.aggregators import KrumAggregator
    g = torch.Generator(device='cuda').manual_seed(n + agg)
    dev = 'cuda' if where == 'device' else 'cpu'
    models = []
    rng = np.random.default_rng(n)
    for i in range(n):
        d = OrderedDict()
        for k, s in KEYS:
            z = (1.0 + 0.3 * i / n) * torch.randn(s, device='cuda',
                                                  generator=g)
            if i >= n - f:
                z = z + 50.0
            d[k] = z.to(dev)
        models.append((int(rng.integers(1, 1000)), d))
    init = OrderedDict((k, torch.randn(s, device='cuda', generator=g).to(dev))
                       for k, s in KEYS)
    res, sel, paths = [], [], []
    for fast in (True, False):
        agg_ = KrumAggregator(model=_Model(init), device='cuda',
                              config=_cfg(f, agg, ignore_weight))
        if not fast:
            agg_._select_on_device = lambda *a, **k: None
        out = agg_.aggregate({'client_feedback': models})
        res.append(out)
        sel.append(list(agg_.last_selection))
        paths.append(agg_.last_pairdist_path)
    # both routes agree on the path too (an uncertified selection leaves
    # the device route for the host's)
    assert paths[0] == paths[1] and paths[0].startswith('mfma')
    assert sel[0] == sel[1]
    assert all(i < n - f for i in sel[0])
    for k in res[0]:
        assert torch.equal(res[0][k], res[1][k]), k
