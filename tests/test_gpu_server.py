"""End to end through the server counterpart (A2/A3) with uploads staged
into HBM on arrival: the reference's own toy-LR course (configs[0] C1,
tests/test_toy_lr.py) captured round by round (tools/capture_toy_lr.py) must
be reproduced bit for bit, and robust rules must accept staged slots."""
from collections import OrderedDict
from types import SimpleNamespace

import json

import numpy as np
import pytest
import torch

import oracle as O
from golden_io import GOLDEN

pytestmark = pytest.mark.gpu


def _cfg(**kw):
    bft = SimpleNamespace(krum_agg_num=kw.get('agg_num', 1),
                          trimmedmean_excluded_ratio=0.2,
                          normbounding_norm_bound=1.0)
    return SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=kw.get('client_num', 1000),
                                 sample_client_rate=1.0),
        aggregator=SimpleNamespace(byzantine_node_num=kw.get('f', 0),
                                   BFT_args=bft),
        asyn=SimpleNamespace(staleness_discount_factor=1.0))


def _rounds():
    with np.load(GOLDEN + '/toy_lr_rounds.npz', allow_pickle=False) as z:
        meta = json.loads(str(z['meta']))
        rounds = []
        for r, rm in enumerate(meta['rounds_meta']):
            ins = [(s, OrderedDict((k, z['r%d|x|%d|%s' % (r, i, k)])
                                   for k in rm['keys']))
                   for i, s in enumerate(rm['sizes'])]
            out = OrderedDict((k, z['r%d|out|%s' % (r, k)])
                              for k in rm['keys'])
            rounds.append((ins, out))
    return meta, rounds


@pytest.mark.parametrize('stage', [True, False])
def test_toy_lr_course_bit_exact(stage):
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.core.workers.server import AggregationServer
    meta, rounds = _rounds()
    assert meta['rounds'] == 20 and meta['test_loss'] < 0.3
    class LR(torch.nn.Module):      # core/lr.py:4-10, toy data 5 features
        def __init__(self):
            super().__init__()
            self.fc = torch.nn.Linear(5, 1)

    model = LR()
    srv = AggregationServer(model, ClientsAvgAggregator(config=_cfg()),
                            sample_client_num=5, stage_on_arrival=stage,
                            keep_history=1)
    for r, (ins, out) in enumerate(rounds):
        for i, (s, d) in enumerate(ins):
            moved = srv.callback_funcs_model_para(
                r, i + 1, (s, OrderedDict((k, torch.from_numpy(v.copy()))
                                          for k, v in d.items())))
            assert moved == (i == len(ins) - 1)
        got = srv.history[-1]
        for k in out:
            assert got[k].cpu().numpy().tobytes() == out[k].tobytes(), (r, k)
        # and the server model now holds the aggregate
        sd = model.state_dict()
        for k in out:
            assert sd[k].numpy().tobytes() == out[k].tobytes(), (r, k)
    assert srv.state == 20


def test_staged_robust_rules_match_unstaged():
    from federatedscope_amd.core.aggregators import (KrumAggregator,
                                                     MedianAggregator)
    from federatedscope_amd.core.workers.ingress import DeviceIngress
    rng = np.random.default_rng(3)
    n = 12
    clients = [(int(rng.integers(1, 50)), OrderedDict(
        [('a', rng.standard_normal((7, 9)).astype(np.float32)),
         ('b', rng.standard_normal(5).astype(np.float32))]))
        for _ in range(n)]
    init = OrderedDict((k, np.zeros_like(v)) for k, v in clients[0][1].items())

    class M(torch.nn.Module):
        def state_dict(self, *a, **kw):
            return OrderedDict((k, torch.from_numpy(v)) for k, v in
                               init.items())

    ing = DeviceIngress(clients[0][1], n)
    staged = [ing.receive(s, OrderedDict((k, torch.from_numpy(v.copy()))
                                         for k, v in d.items()))
              for s, d in clients]
    host = [(s, OrderedDict((k, torch.from_numpy(v.copy()))
                            for k, v in d.items())) for s, d in clients]
    for cls, kw in ((MedianAggregator, {}), (KrumAggregator, {'agg_num': 3})):
        a = cls(model=M(), config=_cfg(f=2, client_num=50, **kw))
        b = cls(model=M(), config=_cfg(f=2, client_num=50, **kw))
        g1 = a.aggregate({'client_feedback': staged})
        g2 = b.aggregate({'client_feedback': host})
        for k in g1:
            assert torch.equal(g1[k].cpu(), g2[k].cpu()), (cls, k)
    want = O.median_aggregate(clients, init)
    g = MedianAggregator(model=M(), config=_cfg(f=2, client_num=50)
                         ).aggregate({'client_feedback': staged})
    for k in want:
        assert g[k].cpu().numpy().tobytes() == want[k].tobytes()


def test_stack_gather_matches_per_key_copies():
    """ClientStack.load_many: device-resident fp32 dicts go through one
    fsagg_gather_rows_f32 launch; rows equal the per-key copies bit for bit,
    absent keys leave the row untouched, and dicts the gather cannot take
    (a non-contiguous or fp16 tensor) fall back to per-key copies."""
    from collections import OrderedDict
    from federatedscope_amd.layout import BucketLayout, ClientStack
    dev = torch.device('cuda')
    g = torch.Generator(device=dev).manual_seed(5)
    shapes = [('a', (3, )), ('b', (2049, )), ('c', (0, )), ('d', (64, 70)),
              ('e', (1, )), ('f', (5000, 3))]
    tmpl = OrderedDict((k, torch.zeros(s)) for k, s in shapes)
    lay = BucketLayout(tmpl)
    n = 9
    models = []
    for i in range(n):
        m = OrderedDict((k, torch.randn(s, device=dev, generator=g))
                        for k, s in shapes)
        if i == 2:
            del m['d']                          # absent key
        if i == 4:
            m['b'] = torch.randn((2049, 2), device=dev,
                                 generator=g)[:, 0]   # non-contiguous
        if i == 6:
            m['f'] = m['f'].half()              # other dtype: converted
        models.append(m)
    fast = ClientStack(lay, n, dev)
    fast.slab.fill_(-3.0)
    fast.load_many(models)
    slow = ClientStack(lay, n, dev)
    slow.slab.fill_(-3.0)
    for i, m in enumerate(models):
        lay.pack_device(m, slow.slab[i])
    torch.cuda.synchronize()
    assert torch.equal(fast.slab, slow.slab)
    o, k = lay.offsets['d'], lay.numels['d']
    assert (fast.slab[2, o:o + k] == -3.0).all()
    for i in (0, 5, 8):
        for key, s in shapes:
            o, k = lay.offsets[key], lay.numels[key]
            assert torch.equal(fast.slab[i, o:o + k],
                               models[i][key].reshape(-1))


def test_large_host_dicts_median_pinned_reuse():
    """~100 MB of host dicts through MedianAggregator: the init
    model is packed into the shared pinned buffer right after the clients'
    DMAs were queued from it, so the stager must wait for them.  Against
    the same clients handed over as device dicts (no pinned staging)."""
    from federatedscope_amd.core.aggregators import MedianAggregator
    g = torch.Generator().manual_seed(12)
    n, shapes = 9, [('w', (2_700_000, )), ('b', (17, ))]
    clients = [(i + 1, OrderedDict((k, torch.randn(s, generator=g))
                                   for k, s in shapes)) for i in range(n)]
    init = OrderedDict((k, torch.randn(s, generator=g)) for k, s in shapes)

    class M(torch.nn.Module):
        def state_dict(self, *a, **kw):
            return init

    host = MedianAggregator(model=M(), config=_cfg(f=1, client_num=50))
    got = host.aggregate({'client_feedback': clients})
    dev = [(s, OrderedDict((k, v.cuda()) for k, v in d.items()))
           for s, d in clients]
    want = MedianAggregator(model=M(), config=_cfg(f=1, client_num=50)
                            ).aggregate({'client_feedback': dev})
    for k in want:
        assert torch.equal(got[k], want[k].cpu()), k
    ref = O.median_aggregate([(s, OrderedDict((k, v.numpy()) for k, v in
                                              d.items())) for s, d in clients],
                             OrderedDict((k, v.numpy())
                                         for k, v in init.items()))
    for k in ref:
        assert got[k].numpy().tobytes() == ref[k].tobytes(), k


def test_staged_with_stale_host_dicts_and_resend():
    """stage_on_arrival with staleness_toleration > 0: the
    round's list mixes staged slots with stale uploads buffered as host
    dicts; a sender that uploads twice in one round keeps its row.  The
    result equals the unstaged server's bit for bit."""
    from federatedscope_amd.core.aggregators import AsynClientsAvgAggregator
    from federatedscope_amd.core.workers.server import AggregationServer
    g = torch.Generator().manual_seed(4)
    shapes = [('w', (300_001, )), ('b', (5, ))]

    def upload():
        return (int(torch.randint(1, 50, (1, ), generator=g)),
                OrderedDict((k, torch.randn(s, generator=g))
                            for k, s in shapes))

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.zeros(300_001))
            self.b = torch.nn.Parameter(torch.zeros(5))

    script = []
    for r in range(3):
        if r > 0:
            script.append((r - 1, 9, upload()))      # stale, tolerated
        script.append((r, 1, upload()))
        script.append((r, 1, upload()))              # resend: overwrites
        for c in (2, 3, 4):
            script.append((r, c, upload()))
    results = []
    for stage in (True, False):
        model = M()
        srv = AggregationServer(model, AsynClientsAvgAggregator(
            model=model, config=_cfg()), sample_client_num=4,
            staleness_toleration=2, stage_on_arrival=stage, keep_history=3)
        for r, c, (s, d) in script:
            srv.callback_funcs_model_para(
                r, c, (s, OrderedDict((k, v.clone()) for k, v in d.items())))
        assert srv.state == 3
        results.append([OrderedDict((k, v.detach().cpu().clone())
                                    for k, v in h.items())
                        for h in srv.history])
    for a, b in zip(*results):
        for k in a:
            assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize('dev', ['cpu', 'cuda'])
def test_server_stages_typed_keys_bit_exact(dev):
    """A model sharing non-trainable keys (share_non_trainable_para: BN's
    int64 num_batches_tracked; here the fedavg_dtypes fixture's int64, fp16,
    bf16 and fp64 keys beside fp32 ones) through stage_on_arrival: the fp32
    keys go into the ingress stack, the others stay typed device copies
    (server.py:966-970 buffers any dict), and the round's FedAvg is
    bit-exact against the reference's output."""
    from golden_io import load_case
    from test_gpu_golden import assert_bit_exact, to_torch
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.core.workers.ingress import StagedUpdate
    from federatedscope_amd.core.workers.server import AggregationServer
    meta, clients, out, _, _ = load_case('fedavg_dtypes')
    keysets = {tuple(d.keys()) for _, d in clients}

    class M(torch.nn.Module):
        def state_dict(self, *a, **kw):
            return OrderedDict()

        def load_state_dict(self, sd, strict=True):
            self.loaded = sd

    srv = AggregationServer(M(), ClientsAvgAggregator(config=_cfg()),
                            sample_client_num=len(clients),
                            stage_on_arrival=True, keep_history=1)
    for i, (s, d) in enumerate(clients):
        srv.callback_funcs_model_para(
            0, i, (s, OrderedDict((k, to_torch(v, dev))
                                  for k, v in d.items())))
        if i < len(clients) - 1 and len(keysets) == 1:
            para = srv.msg_buffer['train'][0][i][1]
            assert isinstance(para, StagedUpdate)
            assert para.typed, 'non-fp32 keys kept beside the slot'
    assert srv.state == 1
    assert_bit_exact(srv.history[-1], out, 'server fedavg_dtypes ' + dev)
    assert srv.ingress.layout.other
