#!/usr/bin/env python3
"""Generate golden vectors for the aggregation path from the REAL reference.

Runs ONLY in the build container (it imports FederatedScope from
/root/reference, which does not exist on the GPU box).  The fixtures it writes
under tests/golden/ are plain data (inputs and the reference's outputs) and are
what travels; this script itself never runs on the GPU box.

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference \
        python3 /root/repo/tools/gen_golden.py

Reference call sites exercised (all under federatedscope/core/aggregators/):
  ClientsAvgAggregator._para_weighted_avg   clients_avg_aggregator.py:60-100
  OnlineClientsAvgAggregator.reset/inc      clients_avg_aggregator.py:115-148
  AsynClientsAvgAggregator.aggregate        asyn_clients_avg_aggregator.py:14-84
  KrumAggregator                            krum_aggregator.py:14-90
  MedianAggregator                          median_aggregator.py:27-52
  TrimmedmeanAggregator                     trimmedmean_aggregator.py:28-57
  BulyanAggregator                          bulyan_aggregator.py:75-106
  NormboundingAggregator                    normbounding_aggregator.py:19-70
  ServerClientsInterpolateAggregator        server_clients_interpolate_aggregator.py:20-30
  FedOptAggregator                          fedopt_aggregator.py:26-44

Inputs are deep-copied before every reference call: the reference mutates
client dicts in place (clients_avg_aggregator.py:69,89; krum_aggregator.py:48-53).
"""
import copy
import json
import os
import sys
from collections import OrderedDict
from types import SimpleNamespace

import numpy as np
import torch

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests',
                   'golden')

from federatedscope.core.aggregators import (  # noqa: E402
    ClientsAvgAggregator, OnlineClientsAvgAggregator, AsynClientsAvgAggregator,
    KrumAggregator, MedianAggregator, TrimmedmeanAggregator, BulyanAggregator,
    NormboundingAggregator, ServerClientsInterpolateAggregator,
    FedOptAggregator)


# --------------------------------------------------------------------------
# helpers
# --------------------------------------------------------------------------
def make_cfg(client_num=1000, ignore_weight=False, use_ss=False, f=0,
             krum_agg_num=1, tm_ratio=0.1, norm_bound=1.0, rate=1.0,
             discount=1.0, fedopt=None):
    bft = SimpleNamespace(krum_agg_num=krum_agg_num,
                          trimmedmean_excluded_ratio=tm_ratio,
                          normbounding_norm_bound=norm_bound)
    fo = fedopt or {'type': 'SGD', 'lr': 1.0}
    return SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=ignore_weight, use_ss=use_ss,
                                 client_num=client_num,
                                 sample_client_rate=rate),
        aggregator=SimpleNamespace(byzantine_node_num=f, BFT_args=bft),
        asyn=SimpleNamespace(staleness_discount_factor=discount),
        fedopt=SimpleNamespace(optimizer=fo, annealing=False))


class DictModel(torch.nn.Module):
    """A module whose state_dict() is exactly the given tensors."""
    def __init__(self, tensors):
        super().__init__()
        self._names = list(tensors.keys())
        for k, v in tensors.items():
            mod_name = k.replace('.', '__')
            if v.dtype.is_floating_point:
                self.register_parameter(mod_name, torch.nn.Parameter(v.clone()))
            else:
                self.register_buffer(mod_name, v.clone())

    def state_dict(self, *a, **kw):
        sd = super().state_dict(*a, **kw)
        return OrderedDict((k.replace('__', '.'), v) for k, v in sd.items())

    def named_parameters(self, *a, **kw):
        for k, v in super().named_parameters(*a, **kw):
            yield k.replace('__', '.'), v


def to_np(t):
    if isinstance(t, str):   # a gRPC upload value: base64 text, as bytes
        return np.frombuffer(t.encode('ascii'), dtype=np.uint8), 'b64'
    t = t.detach().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16), 'bfloat16'
    return t.numpy(), str(t.dtype).replace('torch.', '')


def save_case(name, meta, clients, outputs, init=None, extra=None):
    arrs = {}
    meta = dict(meta)
    meta['n'] = len(clients)
    meta['sizes'] = [int(s) for s, _ in clients]
    meta['keys'] = [list(d.keys()) for _, d in clients]
    meta['dtypes'] = {}
    for i, (_, d) in enumerate(clients):
        for k, v in d.items():
            a, dt = to_np(v)
            arrs['x|%d|%s' % (i, k)] = a
            meta['dtypes']['x|%d|%s' % (i, k)] = dt
    meta['out_keys'] = list(outputs.keys())
    for k, v in outputs.items():
        a, dt = to_np(v)
        arrs['out|' + k] = a
        meta['dtypes']['out|' + k] = dt
    if init is not None:
        meta['init_keys'] = list(init.keys())
        for k, v in init.items():
            a, dt = to_np(v)
            arrs['init|' + k] = a
            meta['dtypes']['init|' + k] = dt
    for k, v in (extra or {}).items():
        arrs['extra|' + k] = np.asarray(v)
    arrs['meta'] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(OUT, name + '.npz'), **arrs)
    print('wrote', name, sum(a.nbytes for a in arrs.values()), 'B')


def rand_clients(rng, n, shapes, dtype=torch.float32, sizes=None, scale=1.0):
    clients = []
    for i in range(n):
        d = OrderedDict()
        for k, shp in shapes.items():
            d[k] = torch.from_numpy(
                (rng.standard_normal(shp) * scale).astype(np.float32)).to(dtype)
        s = int(sizes[i]) if sizes is not None else int(rng.integers(1, 500))
        clients.append((s, d))
    return clients


def run(agg, clients, **info):
    agg_info = {'client_feedback': copy.deepcopy(clients),
                'recover_fun': None}
    agg_info.update(info)
    return agg.aggregate(agg_info)


# --------------------------------------------------------------------------
# cases
# --------------------------------------------------------------------------
def fedavg_cases(rng):
    shapes = OrderedDict([('a.weight', (1, )), ('b.weight', (3, )),
                          ('c.weight', (7, 143)), ('d.bias', (4097, ))])
    for n in (1, 2, 7, 100):
        sh = shapes if n < 100 else OrderedDict([('a.weight', (1, )),
                                                 ('b.weight', (3, )),
                                                 ('c.weight', (1001, ))])
        for iw in (False, True):
            cfg = make_cfg(ignore_weight=iw)
            clients = rand_clients(rng, n, sh)
            out = run(ClientsAvgAggregator(config=cfg), clients)
            save_case('fedavg_n%d_iw%d' % (n, iw), {
                'rule': 'fedavg', 'ignore_weight': iw}, clients, out)

    # heavy-tailed magnitudes + a key missing in one client + zero sizes
    cfg = make_cfg()
    clients = rand_clients(rng, 9, shapes)
    for i, (_, d) in enumerate(clients):
        for k in d:
            d[k] = d[k] * float(10.0 ** rng.integers(-6, 7))
    del clients[4][1]['c.weight']
    clients[6] = (0, clients[6][1])
    out = run(ClientsAvgAggregator(config=cfg), clients)
    save_case('fedavg_missing_key', {'rule': 'fedavg', 'ignore_weight': False},
              clients, out)

    # mixed dtypes: int64, fp16, bf16, fp64 keys (dtype behaviour, A5)
    cfg = make_cfg()
    clients = []
    for i in range(6):
        d = OrderedDict()
        d['w32'] = torch.from_numpy(rng.standard_normal(257).astype(np.float32))
        d['w16'] = torch.from_numpy(
            rng.standard_normal(131).astype(np.float32)).half()
        d['wbf'] = torch.from_numpy(
            rng.standard_normal(131).astype(np.float32)).bfloat16()
        d['w64'] = torch.from_numpy(rng.standard_normal(67))
        d['bn.num_batches_tracked'] = torch.tensor(int(rng.integers(0, 10**6)),
                                                   dtype=torch.long)
        d['cnt'] = torch.from_numpy(rng.integers(-1000, 1000, size=33))
        clients.append((int(rng.integers(1, 300)), d))
    out = run(ClientsAvgAggregator(config=cfg), clients)
    save_case('fedavg_dtypes', {'rule': 'fedavg', 'ignore_weight': False},
              clients, out)

    # ServerClientsInterpolate (pFedMe path): two chained weighted averages
    for beta in (1.0, 0.7):
        cfg = make_cfg()
        clients = rand_clients(rng, 5, shapes)
        init = OrderedDict((k, torch.from_numpy(
            rng.standard_normal(s).astype(np.float32))) for k, s in
                           shapes.items())
        agg = ServerClientsInterpolateAggregator(model=DictModel(init),
                                                 config=cfg, beta=beta)
        out = run(agg, clients)
        save_case('interp_beta%s' % str(beta).replace('.', 'p'), {
            'rule': 'interpolate', 'beta': beta}, clients, out, init=init)


def asyn_cases(rng):
    shapes = OrderedDict([('w', (3, 129)), ('b', (5, ))])
    for factor in (0.5, 1.0):
        for iw in (False, True):
            cfg = make_cfg(ignore_weight=iw, discount=factor)
            n = 8
            clients = rand_clients(rng, n, shapes)
            stal = [(i + 1, int(rng.integers(0, 3))) for i in range(n)]
            init = OrderedDict((k, torch.from_numpy(
                rng.standard_normal(s).astype(np.float32))) for k, s in
                               shapes.items())
            agg = AsynClientsAvgAggregator(model=DictModel(init), config=cfg)
            out = run(agg, clients, staleness=stal)
            save_case('asyn_f%s_iw%d' % (str(factor).replace('.', 'p'), iw), {
                'rule': 'asyn', 'factor': factor, 'ignore_weight': iw,
                'staleness': [s for _, s in stal]}, clients, out, init=init)


def online_cases(rng):
    shapes = OrderedDict([('w', (17, 31)), ('b', (31, ))])
    init = OrderedDict((k, torch.from_numpy(
        rng.standard_normal(s).astype(np.float32))) for k, s in shapes.items())
    agg = OnlineClientsAvgAggregator(model=DictModel(init), config=make_cfg())
    agg.reset()
    clients = rand_clients(rng, 11, shapes)
    for s, d in copy.deepcopy(clients):
        agg.inc((s, d))
    out = agg.aggregate({})
    save_case('online_n11', {'rule': 'online'}, clients, out, init=init)


def krum_cases(rng):
    shapes = OrderedDict([('conv.w', (4, 3, 5)), ('fc.w', (3, 300)),
                          ('fc.b', (3, ))])
    # (n, f, agg_num, client_num for the ctor assert)
    for n, f, agg_num in ((7, 1, 1), (12, 2, 3), (12, 2, 5), (50, 10, 1),
                          (50, 10, 5), (50, 10, 30), (10, 10, 1)):
        cfg = make_cfg(client_num=max(2 * f + 3, 50), f=f,
                       krum_agg_num=agg_num)
        base = OrderedDict((k, rng.standard_normal(s).astype(np.float32))
                           for k, s in shapes.items())
        clients = []
        byz = set(rng.choice(n, size=min(f, n // 3), replace=False).tolist())
        for i in range(n):
            d = OrderedDict()
            for k, s in shapes.items():
                if i in byz:
                    v = 0.1 + 0.5 * rng.standard_normal(s)
                else:
                    v = base[k] + 0.05 * (1 + 0.05 * i) * \
                        rng.standard_normal(s)
                d[k] = torch.from_numpy(v.astype(np.float32))
            clients.append((int(rng.integers(1, 500)), d))
        init = OrderedDict((k, torch.from_numpy(
            rng.standard_normal(s).astype(np.float32))) for k, s in
                           shapes.items())
        agg = KrumAggregator(model=DictModel(init), config=cfg)
        paras = copy.deepcopy([c[1] for c in clients])
        scores = agg._calculate_score(paras)
        order = torch.sort(scores)[1].numpy()
        # the distance matrix the scores come from (same reference code)
        paras = copy.deepcopy([c[1] for c in clients])
        D = np.zeros((n, n), dtype=np.float32)
        for a in range(n):
            for b in range(a, n):
                D[a, b] = np.inf if a == b else float(
                    agg._calculate_distance(paras[a], paras[b]))
                D[b, a] = D[a, b]
        out = run(agg, clients)
        save_case('krum_n%d_f%d_a%d' % (n, f, agg_num), {
            'rule': 'krum', 'f': f, 'agg_num': agg_num}, clients, out,
                  init=init, extra={'D': D, 'scores': scores.numpy(),
                                    'order': order})


def order_stat_cases(rng):
    for n in (5, 6, 7, 50, 51, 200):
        for P in (48, 51):
            shapes = OrderedDict([('w', (P, )), ('v', (2, 7))])
            clients = rand_clients(rng, n, shapes)
            # outliers (x100) on 10% of clients, like configs C5
            for i in rng.choice(n, size=max(1, n // 10), replace=False):
                for k in clients[i][1]:
                    clients[i][1][k] = clients[i][1][k] * 100.0
            # exact ties in one coordinate column
            for i in range(n):
                clients[i][1]['w'][3] = float(i % 3)
            init = OrderedDict((k, torch.from_numpy(
                rng.standard_normal(s).astype(np.float32))) for k, s in
                               shapes.items())
            cfg = make_cfg(client_num=1000, f=1, tm_ratio=0.2)
            out = run(MedianAggregator(model=DictModel(init), config=cfg),
                      clients)
            # trimmed-mean outputs for several ratios share the inputs
            extra = {}
            for ratio in (0.1, 0.2, 0.45):
                cfg = make_cfg(client_num=1000, f=1, tm_ratio=ratio)
                tm = run(
                    TrimmedmeanAggregator(model=DictModel(init), config=cfg),
                    clients)
                for k, v in tm.items():
                    extra['tm|%s|%s' % (ratio, k)] = v.numpy()
            save_case('orderstat_n%d_p%d' % (n, P), {
                'rule': 'median', 'tm_ratios': [0.1, 0.2, 0.45]}, clients,
                      out, init=init, extra=extra)


def order_stat_nonfinite_cases(rng):
    """±inf / NaN columns through MedianAggregator and TrimmedmeanAggregator
    (k = 0 and k >= 1), so the oracle's non-finite rule is pinned to the
    reference's own outputs."""
    for n in (9, 20):
        P = 8
        shapes = OrderedDict([('w', (P, ))])
        clients = rand_clients(rng, n, shapes)
        W = np.stack([c[1]['w'].numpy() for c in clients])
        W[0, 0] = np.nan
        W[0, 1] = np.inf
        W[0, 2] = -np.inf
        W[1, 3] = np.inf
        W[2, 3] = -np.inf
        W[3:, 5] = np.inf
        for i in range(n):
            clients[i][1]['w'] = torch.from_numpy(W[i].copy())
        init = OrderedDict([('w', torch.zeros(P))])
        cfg = make_cfg(client_num=1000, f=1, tm_ratio=0.2)
        out = run(MedianAggregator(model=DictModel(init), config=cfg),
                  clients)
        extra = {}
        for ratio in (0.0, 0.1, 0.2):
            cfg = make_cfg(client_num=1000, f=1, tm_ratio=ratio)
            tm = run(TrimmedmeanAggregator(model=DictModel(init), config=cfg),
                     clients)
            for k, v in tm.items():
                extra['tm|%s|%s' % (ratio, k)] = v.numpy()
        save_case('orderstat_nonfinite_n%d' % n, {
            'rule': 'median', 'tm_ratios': [0.0, 0.1, 0.2]}, clients, out,
                  init=init, extra=extra)


def bulyan_cases(rng):
    shapes = OrderedDict([('w', (3, 41)), ('b', (9, ))])
    for n, f, rate in ((11, 2, 1.0), (20, 4, 0.5), (40, 9, 1.0)):
        cfg = make_cfg(client_num=4 * f + 3, f=f, rate=rate)
        clients = rand_clients(rng, n, shapes, scale=0.1)
        for i in rng.choice(n, size=f, replace=False):
            for k in clients[i][1]:
                clients[i][1][k] = clients[i][1][k] + 3.0
        init = OrderedDict((k, torch.from_numpy(
            rng.standard_normal(s).astype(np.float32))) for k, s in
                           shapes.items())
        agg = BulyanAggregator(model=DictModel(init), config=cfg)
        scores = agg._calculate_score(copy.deepcopy([c[1] for c in clients]))
        order = torch.sort(scores)[1].numpy()
        out = run(agg, clients)
        save_case('bulyan_n%d_f%d' % (n, f), {
            'rule': 'bulyan', 'f': f, 'rate': rate}, clients, out, init=init,
                  extra={'scores': scores.numpy(), 'order': order})


def normbound_cases(rng):
    shapes = OrderedDict([('w', (7, 33)), ('b', (7, )), ('bn.x', (4, ))])
    for bound in (0.5, 5.0, 1e6):
        cfg = make_cfg(norm_bound=bound)
        clients = rand_clients(rng, 9, shapes, scale=0.3)
        init = OrderedDict((k, torch.from_numpy(
            rng.standard_normal(s).astype(np.float32))) for k, s in
                           shapes.items())
        agg = NormboundingAggregator(model=DictModel(init), config=cfg)
        out = run(agg, clients)
        save_case('normbound_%g' % bound, {
            'rule': 'normbounding', 'bound': bound}, clients, out, init=init)


def fedopt_cases(rng):
    shapes = OrderedDict([('w', (5, 21)), ('b', (5, ))])
    for opt in ({'type': 'SGD', 'lr': 1.0}, {'type': 'SGD', 'lr': 0.5,
                                               'momentum': 0.9},
                {'type': 'Adam', 'lr': 0.01}):
        cfg = make_cfg(fedopt=opt)
        init = OrderedDict((k, torch.from_numpy(
            rng.standard_normal(s).astype(np.float32))) for k, s in
                           shapes.items())
        agg = FedOptAggregator(config=cfg, model=DictModel(init))
        rounds = []
        outs = []
        for r in range(3):
            clients = rand_clients(rng, 4, shapes)
            rounds.append(clients)
            # state_dict() shares storage with the parameters the next
            # rounds update in place: snapshot it
            outs.append(OrderedDict((k, v.detach().clone())
                                    for k, v in run(agg, clients).items()))
        # save each round as its own case sharing the optimizer state chain
        for r in range(3):
            save_case('fedopt_%s_%d' % (opt['type'] + ('m' if 'momentum' in
                                                       opt else ''), r), {
                'rule': 'fedopt', 'opt': opt, 'round': r}, rounds[r], outs[r],
                      init=init if r == 0 else None)


def normbound_missing_key_cases(rng):
    """Clients whose keys differ from the server model's
    (normbounding_aggregator.py:49-70): the norm runs over the server keys
    a client holds, and a scaled client is rebuilt from a deepcopy of the
    server model — keys it lacks come back as the SERVER's values."""
    shapes = OrderedDict([('w', (7, 33)), ('b', (7, )), ('bn.x', (4, ))])
    for tag, bound in (('scaled', 0.5), ('mixed', 2.0), ('none', 1e6)):
        for variant in ('peer', 'first', 'extra'):
            cfg = make_cfg(norm_bound=bound)
            clients = rand_clients(rng, 9, shapes, scale=0.3)
            # a spread of norms so that 'mixed' scales some clients only
            for i, (_, d) in enumerate(clients):
                for k in d:
                    d[k] = d[k] * float(0.2 + 0.25 * i)
            if variant == 'peer':
                del clients[3][1]['b']
                del clients[6][1]['bn.x']
            elif variant == 'first':
                del clients[0][1]['bn.x']
                del clients[4][1]['w']
            else:   # a key the server model does not have
                clients[5][1]['extra.w'] = torch.from_numpy(
                    rng.standard_normal(5).astype(np.float32))
                del clients[2][1]['b']
            init = OrderedDict((k, torch.from_numpy(
                rng.standard_normal(s).astype(np.float32))) for k, s in
                               shapes.items())
            agg = NormboundingAggregator(model=DictModel(init), config=cfg)
            out = run(agg, clients)
            save_case('normbound_keys_%s_%s' % (tag, variant), {
                'rule': 'normbounding', 'bound': bound}, clients, out,
                      init=init)


def online_dtype_cases(rng):
    """OnlineClientsAvgAggregator.inc with non-fp32 keys
    (clients_avg_aggregator.py:125-142): ATen promotes — an int64 buffer's
    running mean becomes fp32 at the first division, an fp16 upload of an
    fp32 key is multiplied in fp16, an fp64 upload promotes the key."""
    init = OrderedDict([
        ('w', torch.from_numpy(rng.standard_normal((5, 7)).astype(
            np.float32))),
        ('n', torch.tensor(int(rng.integers(0, 100)), dtype=torch.long)),
        ('h', torch.from_numpy(rng.standard_normal(6).astype(
            np.float32)).half()),
        ('c', torch.from_numpy(rng.integers(-50, 50, 4))),
    ])
    agg = OnlineClientsAvgAggregator(model=DictModel(init),
                                     config=make_cfg())
    agg.reset()
    clients = []
    for i in range(6):
        d = OrderedDict()
        wv = rng.standard_normal((5, 7)).astype(np.float32)
        d['w'] = torch.from_numpy(wv).half() if i % 3 == 1 else \
            torch.from_numpy(wv)
        d['n'] = torch.tensor(int(rng.integers(0, 10**6)), dtype=torch.long)
        hv = rng.standard_normal(6)
        d['h'] = torch.from_numpy(hv) if i == 4 else \
            torch.from_numpy(hv.astype(np.float32)).half() if i % 2 else \
            torch.from_numpy(hv.astype(np.float32))
        if i != 2:
            d['c'] = torch.from_numpy(rng.integers(-1000, 1000, 4))
        clients.append((int(rng.integers(1, 300)), d))
    for s, d in copy.deepcopy(clients):
        agg.inc((s, d))
    out = agg.aggregate({})
    # the server model's state_dict order (parameters, then buffers) is
    # the order the reference iterates: save init in that order
    order = list(DictModel(init).state_dict().keys())
    save_case('online_dtypes_n6', {'rule': 'online'}, clients, out,
              init=OrderedDict((k, init[k]) for k in order))


def fedopt_more_cases(rng):
    """FedOpt configs the device path first lacked: Adam(amsgrad) and a
    float64 server model (fedopt_aggregator.py:26-44 runs any
    torch.optim config)."""
    shapes = OrderedDict([('w', (5, 21)), ('b', (5, ))])
    for tag, opt, dt in (
            ('AdamAms', {'type': 'Adam', 'lr': 0.01, 'amsgrad': True},
             torch.float32),
            ('SGDm64', {'type': 'SGD', 'lr': 0.5, 'momentum': 0.9,
                        'weight_decay': 0.01}, torch.float64),
            ('Adam64', {'type': 'Adam', 'lr': 0.01}, torch.float64)):
        cfg = make_cfg(fedopt=opt)
        init = OrderedDict((k, torch.from_numpy(
            rng.standard_normal(s)).to(dt)) for k, s in shapes.items())
        agg = FedOptAggregator(config=cfg, model=DictModel(init))
        rounds, outs = [], []
        for r in range(3):
            clients = rand_clients(rng, 4, shapes, dtype=dt)
            rounds.append(clients)
            outs.append(OrderedDict((k, v.detach().clone())
                                    for k, v in run(agg, clients).items()))
        for r in range(3):
            save_case('fedopt_%s_%d' % (tag, r), {
                'rule': 'fedopt', 'opt': opt, 'round': r}, rounds[r],
                      outs[r], init=init if r == 0 else None)


def fedopt_round3_cases(rng):
    """FedOpt with every torch.optim class the device step implements
    (optimizer_builder.py:53-56 builds any by name): AdamW, Adagrad,
    RMSprop (plain, momentum, centered), weight decay and maximize; one
    float64 chain; and a chain whose clients drop a parameter in round 1
    (torch.optim keeps per-parameter state and steps)."""
    shapes = OrderedDict([('w', (5, 21)), ('b', (5, ))])
    for tag, opt, dt, drop in (
            ('AdamW', {'type': 'AdamW', 'lr': 0.01}, torch.float32, None),
            ('AdamWams', {'type': 'AdamW', 'lr': 0.02, 'weight_decay': 0.1,
                          'amsgrad': True}, torch.float32, None),
            ('Adagrad', {'type': 'Adagrad', 'lr': 0.1}, torch.float32, None),
            ('Adagradx', {'type': 'Adagrad', 'lr': 0.1, 'lr_decay': 0.05,
                          'weight_decay': 0.01,
                          'initial_accumulator_value': 0.1}, torch.float32,
             None),
            ('RMSprop', {'type': 'RMSprop', 'lr': 0.01}, torch.float32, None),
            ('RMSpropmc', {'type': 'RMSprop', 'lr': 0.01, 'momentum': 0.9,
                           'centered': True, 'weight_decay': 0.01},
             torch.float32, None),
            ('SGDmax', {'type': 'SGD', 'lr': 0.5, 'momentum': 0.9,
                        'maximize': True}, torch.float32, None),
            ('RMSprop64', {'type': 'RMSprop', 'lr': 0.01, 'momentum': 0.5},
             torch.float64, None),
            ('Adamdrop', {'type': 'Adam', 'lr': 0.01}, torch.float32, 'b')):
        cfg = make_cfg(fedopt=opt)
        init = OrderedDict((k, torch.from_numpy(
            rng.standard_normal(s)).to(dt)) for k, s in shapes.items())
        agg = FedOptAggregator(config=cfg, model=DictModel(init))
        rounds, outs = [], []
        for r in range(3):
            clients = rand_clients(rng, 4, shapes, dtype=dt)
            if drop and r == 1:
                for _, d in clients:
                    del d[drop]
            rounds.append(clients)
            outs.append(OrderedDict((k, v.detach().clone())
                                    for k, v in run(agg, clients).items()))
        for r in range(3):
            save_case('fedopt_%s_%d' % (tag, r), {
                'rule': 'fedopt', 'opt': opt, 'round': r}, rounds[r],
                      outs[r], init=init if r == 0 else None)


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(1)  # fed_runner.py:297-299
    if sys.argv[1:] == ['nonfinite']:  # added later: its own seed
        order_stat_nonfinite_cases(np.random.default_rng(20261016))
        return 0
    if sys.argv[1:] == ['round3']:     # round 3 cases: their own seed
        fedopt_round3_cases(np.random.default_rng(20261018))
        return 0
    if sys.argv[1:] == ['round2']:     # round 2 cases: their own seed
        rng = np.random.default_rng(20261017)
        normbound_missing_key_cases(rng)
        online_dtype_cases(rng)
        fedopt_more_cases(rng)
        return 0
    rng = np.random.default_rng(20261015)
    fedavg_cases(rng)
    asyn_cases(rng)
    online_cases(rng)
    krum_cases(rng)
    order_stat_cases(rng)
    bulyan_cases(rng)
    normbound_cases(rng)
    fedopt_cases(rng)


if __name__ == '__main__':
    sys.exit(main())
