"""GPU parity: the drop-in aggregators (HIP path through libfsagg's C ABI)
against the reference's own outputs (tests/golden, generated from
FederatedScope v0.3.0 by tools/gen_golden.py) and the CPU oracle.

Bars: FedAvg / async / online / interpolation / median / Krum average
bit-exact; Krum & Bulyan selected indices exact; trimmed mean, Bulyan and
norm bounding within the tolerance stated per test.
"""
from collections import OrderedDict
from types import SimpleNamespace

import numpy as np
import pytest
import torch

import oracle as O
import trimmed_bounds as TB
from golden_io import case_names, load_case

pytestmark = pytest.mark.gpu



# FedOpt golden chains (tools/gen_golden.py): every torch.optim class the
# device step implements, weight decay, maximize, float64, a dropped key
FEDOPT_CHAINS = ['SGD', 'SGDm', 'Adam', 'AdamAms', 'SGDm64', 'Adam64',
                 'AdamW', 'AdamWams', 'Adagrad', 'Adagradx', 'RMSprop',
                 'RMSpropmc', 'SGDmax', 'RMSprop64', 'Adamdrop']

def to_torch(a, device='cuda'):
    if isinstance(a, O.BF16):
        return torch.from_numpy(a.bits.view(np.int16).copy()).view(
            torch.bfloat16).to(device)
    return torch.from_numpy(np.array(a, copy=True)).to(device)


def to_np(t):
    t = t.detach().cpu()
    if t.dtype == torch.bfloat16:
        return O.BF16(t.view(torch.int16).numpy().view(np.uint16))
    return t.numpy()


def feedback(clients, device='cuda'):
    return [(s, OrderedDict((k, to_torch(v, device)) for k, v in d.items()))
            for s, d in clients]


def cfg(**kw):
    bft = SimpleNamespace(krum_agg_num=kw.get('agg_num', 1),
                          trimmedmean_excluded_ratio=kw.get('ratio', 0.1),
                          normbounding_norm_bound=kw.get('bound', 1.0))
    return SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=kw.get('iw', False),
                                 use_ss=False,
                                 client_num=kw.get('client_num', 1000),
                                 sample_client_rate=kw.get('rate', 1.0)),
        aggregator=SimpleNamespace(byzantine_node_num=kw.get('f', 0),
                                   BFT_args=bft),
        asyn=SimpleNamespace(staleness_discount_factor=kw.get('factor', 1.0)))


class DictModel(torch.nn.Module):
    def __init__(self, sd):
        super().__init__()
        self._sd = OrderedDict((k, to_torch(v, 'cpu')) for k, v in sd.items())

    def state_dict(self, *a, **kw):
        return OrderedDict((k, v.clone()) for k, v in self._sd.items())


def bits(a):
    """Bytes of every element, NaNs canonicalised (a NaN's sign/payload
    depends on the ISA that produced it: x86 gives 0xFFC00000 for
    inf - inf, gfx950 0x7FC00000)."""
    if isinstance(a, O.BF16):
        return a.bits.tobytes()
    a = np.ascontiguousarray(a)
    if a.dtype.kind == 'f' and np.isnan(a).any():
        a = np.where(np.isnan(a), np.asarray(np.nan, a.dtype), a)
    return a.tobytes()


def assert_bit_exact(got, want, what):
    assert list(got.keys()) == list(want.keys()), what
    for k in want:
        g = to_np(got[k])
        w = want[k]
        if not isinstance(w, O.BF16):
            assert g.dtype == np.asarray(w).dtype, (what, k, g.dtype)
            assert g.shape == np.asarray(w).shape, (what, k)
        assert bits(g) == bits(w), (what, k)


@pytest.mark.parametrize('name', case_names('fedavg_'))
def test_fedavg(name):
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    meta, clients, out, _, _ = load_case(name)
    for dev in ('cuda', 'cpu'):   # device-resident and host-dict inputs
        agg = ClientsAvgAggregator(config=cfg(iw=meta['ignore_weight']))
        got = agg.aggregate({'client_feedback': feedback(clients, dev),
                             'recover_fun': None})
        assert_bit_exact(got, out, name + '/' + dev)
        assert all(v.device.type == dev for v in got.values())


@pytest.mark.parametrize('name', case_names('interp_'))
def test_interpolate(name):
    from federatedscope_amd.core.aggregators import \
        ServerClientsInterpolateAggregator
    meta, clients, out, init, _ = load_case(name)
    agg = ServerClientsInterpolateAggregator(model=DictModel(init),
                                             config=cfg(), beta=meta['beta'])
    got = agg.aggregate({'client_feedback': feedback(clients)})
    assert_bit_exact(got, out, name)


@pytest.mark.parametrize('name', case_names('asyn_'))
def test_asyn(name):
    from federatedscope_amd.core.aggregators import AsynClientsAvgAggregator
    meta, clients, out, init, _ = load_case(name)
    agg = AsynClientsAvgAggregator(model=DictModel(init), config=cfg(
        iw=meta['ignore_weight'], factor=meta['factor']))
    got = agg.aggregate({
        'client_feedback': feedback(clients),
        'recover_fun': None,
        'staleness': [(i, s) for i, s in enumerate(meta['staleness'])]
    })
    assert_bit_exact(got, out, name)


@pytest.mark.parametrize('name', case_names('online_'))
def test_online(name):
    from federatedscope_amd.core.aggregators import \
        OnlineClientsAvgAggregator
    meta, clients, out, init, _ = load_case(name)
    agg = OnlineClientsAvgAggregator(model=DictModel(init), config=cfg())
    agg.reset()
    for s, d in feedback(clients):
        agg.inc((s, d))
    assert_bit_exact(agg.aggregate({}), out, name)


@pytest.mark.parametrize('name', case_names('krum_'))
def test_krum(name):
    from federatedscope_amd.core.aggregators import KrumAggregator
    meta, clients, out, init, extra = load_case(name)
    agg = KrumAggregator(model=DictModel(init), config=cfg(
        f=meta['f'], agg_num=meta['agg_num'],
        client_num=max(2 * meta['f'] + 3, 50)))
    fb = feedback(clients)
    D, _ = agg.distance_matrix(fb)
    n = len(clients)
    off = ~np.eye(n, dtype=bool)
    # per-key sums in fp32 chunks + fp64 across chunks vs ATen's fp32 dist
    np.testing.assert_allclose(D.numpy()[off], extra['D'][off], rtol=1e-5)
    assert np.isinf(np.diag(D.numpy())).all()
    got = agg.aggregate({'client_feedback': fb})
    assert agg.last_selection == [int(i) for i in
                                  extra['order'][:meta['agg_num']]]
    assert_bit_exact(got, out, name)


@pytest.mark.parametrize('name', case_names('orderstat_'))
def test_median_and_trimmed(name):
    from federatedscope_amd.core.aggregators import (MedianAggregator,
                                                     TrimmedmeanAggregator)
    meta, clients, out, init, extra = load_case(name)
    fb = feedback(clients)
    got = MedianAggregator(model=DictModel(init), config=cfg(f=1)).aggregate(
        {'client_feedback': fb})
    assert_bit_exact(got, out, name)
    eps = np.finfo(np.float32).eps
    for ratio in meta['tm_ratios']:
        got = TrimmedmeanAggregator(model=DictModel(init), config=cfg(
            f=1, ratio=ratio)).aggregate({'client_feedback': fb})
        k = int(len(clients) * ratio)
        ours = O.add_init(init, O.trimmed_mean_update(clients, k))
        div = len(clients) - 2 * k
        for key in got:
            g = to_np(got[key]).astype(np.float64)
            ref = extra['tm|%s|%s' % (ratio, key)]
            # non-finite columns: the reference's NaN / ±inf exactly
            fin = np.isfinite(ref)
            assert np.array_equal(np.isnan(g), np.isnan(ref)), (name, ratio)
            assert np.array_equal(g[np.isinf(ref)], ref[np.isinf(ref)])
            T = np.stack([np.asarray(d[key], dtype=np.float64).reshape(-1)
                          for _, d in clients])[:, fin.reshape(-1)]
            g, ref, o = g[fin], ref[fin], np.asarray(ours[key])[fin]
            ini = np.asarray(init[key])[fin]
            tag = '%s|tm%s|%s' % (name, ratio, key)
            # vs the reference (ATen cascade sum): §8(c)'s contract
            TB.check_vs_ref(tag, g, ref, T, div)
            # vs the oracle's fp64 middle sum: the regression bound
            TB.check_vs_oracle(tag, g, o, T, div, init=ini)


@pytest.mark.parametrize('name', case_names('bulyan_'))
def test_bulyan(name):
    from federatedscope_amd.core.aggregators import BulyanAggregator
    meta, clients, out, init, extra = load_case(name)
    agg = BulyanAggregator(model=DictModel(init), config=cfg(
        f=meta['f'], rate=meta['rate'], client_num=4 * meta['f'] + 3))
    got = agg.aggregate({'client_feedback': feedback(clients)})
    keep = len(clients) - int(2 * meta['rate'] * meta['f'])
    sel = [int(i) for i in extra['order'][:keep]]
    assert agg.last_selection == sel
    # the output is the trimmed mean of the selected clients
    # (bulyan_aggregator.py:95-106: cat-sum / gamma, then init + update):
    # the same bounds as the trimmed mean — the reference's own rounding
    # bound over the selected clients, and a few ulps of the oracle's fp64
    # middle sum
    k = int(meta['rate'] * meta['f'])
    chosen = [clients[i] for i in sel]
    ours, osel = O.bulyan_aggregate(clients, meta['f'], meta['rate'], init)
    assert osel == sel
    for key in out:
        g = to_np(got[key]).astype(np.float64).reshape(-1)
        ref = out[key].astype(np.float64).reshape(-1)
        o = np.asarray(ours[key]).reshape(-1)
        ini = np.asarray(init[key], dtype=np.float64).reshape(-1)
        T = np.stack([np.asarray(d[key], dtype=np.float64).reshape(-1)
                      for _, d in chosen])
        tag = '%s|%s' % (name, key)
        TB.check_vs_ref(tag, g, ref, T, keep - 2 * k)
        TB.check_vs_oracle(tag, g, o, T, keep - 2 * k, init=ini)


@pytest.mark.parametrize('name', case_names('normbound_'))
def test_normbounding(name):
    from federatedscope_amd.core.aggregators import NormboundingAggregator
    meta, clients, out, init, _ = load_case(name)
    agg = NormboundingAggregator(model=DictModel(init),
                                 config=cfg(bound=meta['bound']))
    got = agg.aggregate({'client_feedback': feedback(clients)})
    # vs the oracle (the correctly rounded fp32 norm, the reference's rate
    # and weighted-sum arithmetic): bit-exact
    ours = O.normbounding_aggregate(clients, meta['bound'], init)
    for key in out:
        assert to_np(got[key]).tobytes() == \
            np.asarray(ours[key], dtype=np.float32).tobytes(), (name, key)
    # vs the reference: its fp32 torch.norm may differ from the correctly
    # rounded norm by its summation error, at most (log2(m) + 2)·ε over m
    # squares (ATen's cascade sum); the rate carries that plus its two
    # roundings into each scaled client, and the sums round differently
    # from there (4ε of the result)
    eps = np.finfo(np.float32).eps
    m = max(sum(int(np.prod(np.shape(d[k]))) for k in init if k in d)
            for _, d in clients)
    eta = (np.ceil(np.log2(max(m, 2))) + 4) * eps
    sizes = np.array([s for s, _ in clients], dtype=np.float64)
    w = sizes / sizes.sum()
    for key in out:
        g = to_np(got[key]).astype(np.float64)
        ref = out[key].astype(np.float64)
        mag = sum(wi * np.abs(np.asarray(d.get(key, 0.0), dtype=np.float64))
                  for wi, (_, d) in zip(w, clients))
        assert (np.abs(g - ref) <= eta * mag + 4 * eps * np.abs(ref) +
                1e-30).all(), (name, key)


class ParamModel(torch.nn.Module):
    """Module whose parameters are the fixture's init tensors."""
    def __init__(self, sd):
        super().__init__()
        for k, v in sd.items():
            self.register_parameter(k, torch.nn.Parameter(to_torch(v, 'cpu')))


@pytest.mark.parametrize('model_dev', ['cpu', 'cuda'])
@pytest.mark.parametrize('opt', FEDOPT_CHAINS)
def test_fedopt_chain(opt, model_dev):
    """Three chained FedOpt rounds (optimizer state carried across rounds)
    against the reference (torch.optim on CPU): tolerance-pinned, the
    reference's vectorised fmadd arithmetic being ISA-dependent.  A model on
    the GPU has its fp32 parameters stepped in place."""
    from federatedscope_amd.core.aggregators import FedOptAggregator
    metas = [load_case('fedopt_%s_%d' % (opt, r)) for r in range(3)]
    meta0, _, _, init, _ = metas[0]
    c = cfg()
    c.fedopt = SimpleNamespace(optimizer=dict(meta0['opt']), annealing=False)
    model = ParamModel(init).to(model_dev)
    agg = FedOptAggregator(config=c, model=model)
    for r, (meta, clients, out, _, _) in enumerate(metas):
        got = agg.aggregate({'client_feedback': feedback(clients),
                             'recover_fun': None})
        assert list(got.keys()) == list(out.keys())
        f64 = opt.endswith('64')
        for k in out:
            # a few ulps of the O(1) parameters: ATen's CPU Adam
            # (lerp/addcmul/addcdiv, vectorised fmadd) rounds differently
            assert to_np(got[k]).dtype == out[k].dtype
            np.testing.assert_allclose(to_np(got[k]), out[k],
                                       rtol=1e-12 if f64 else 2e-6,
                                       atol=1e-14 if f64 else 4e-7,
                                       err_msg='%s r%d %s' % (opt, r, k))


def test_fedopt_use_ss_routes_through_secret_sharing():
    """FedOpt's super().aggregate() (fedopt_aggregator.py:30) is the
    secret-sharing average when federate.use_ss: the optimizer then steps
    toward the recovered average."""
    from federatedscope_amd.core.aggregators import (ClientsAvgAggregator,
                                                     FedOptAggregator)
    meta, clients, out, _, _ = load_case('ss_n3')

    class Rec:
        mod_number = int(meta['mod_number'])
        maximum = int(meta['maximum'])
        epsilon = meta['epsilon']

        def __call__(self, x):
            raise AssertionError('not called on the device path')

    init = OrderedDict((k, np.zeros(np.asarray(v).shape, np.float32))
                       for k, v in out.items())

    class ParamModel(torch.nn.Module):   # dotted parameter names
        def __init__(self, sd):
            super().__init__()
            for k, v in sd.items():
                self.register_parameter(k.replace('.', '__'),
                                        torch.nn.Parameter(to_torch(v,
                                                                    'cpu')))

        def named_parameters(self, *a, **kw):
            for k, v in super().named_parameters(*a, **kw):
                yield k.replace('__', '.'), v

        def state_dict(self, *a, **kw):
            return OrderedDict((k.replace('__', '.'), v) for k, v in
                               super().state_dict(*a, **kw).items())

    c = cfg()
    c.federate.use_ss = True
    c.fedopt = SimpleNamespace(optimizer={'type': 'SGD', 'lr': 1.0},
                               annealing=False)
    agg = FedOptAggregator(config=c, model=ParamModel(init))
    got = agg.aggregate({'client_feedback': clients, 'recover_fun': Rec()})
    # SGD with lr 1 from a zero model lands exactly on the average:
    # 0 - (0 - avg) = avg
    for k in out:
        np.testing.assert_array_equal(to_np(got[k]), np.asarray(out[k]))
