#!/usr/bin/env python3
"""The §8(f) server paths next to the reduction, on one GPU, device dicts:

  online   OnlineClientsAvgAggregator.inc (clients_avg_aggregator.py:103-148)
           per upload of a 25M fp32 model: one fsagg_online_inc_f32 pass,
           12 B per parameter (m read, x read, m written).
  fedopt   FedOptAggregator.aggregate (fedopt_aggregator.py:9-44) with Adam
           over 100 clients x 25M: the FedAvg reduction plus the fused
           optimizer step; reported next to a plain ClientsAvgAggregator
           call on the same dicts (the step's own cost is the difference).

One JSON line per path: median wall time of synchronised calls and the
algorithmic rate.  GPU only."""
import json
import os
import statistics
import sys
import time
from collections import OrderedDict
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

P = 25_000_000


def cfg():
    return SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=1000, sample_client_rate=1.0),
        aggregator=SimpleNamespace(byzantine_node_num=0))


class ParamModel(torch.nn.Module):
    def __init__(self, sd):
        super().__init__()
        for k, v in sd.items():
            self.register_parameter(k, torch.nn.Parameter(v))


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    from federatedscope_amd.core.aggregators import (ClientsAvgAggregator,
                                                     FedOptAggregator)
    from federatedscope_amd.core.aggregators.clients_avg_aggregator import \
        OnlineClientsAvgAggregator
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(5)
    which = sys.argv[1:] or ['online', 'fedopt']
    if 'online' in which:
        init = OrderedDict(w=torch.zeros(P, device=dev))
        agg = OnlineClientsAvgAggregator(model=ParamModel(init), device=dev,
                                         src_device=dev, config=cfg())
        agg.reset()
        up = OrderedDict(w=torch.randn(P, device=dev, generator=g))
        t = timed(lambda: agg.inc((7, up)), reps=20)
        print(json.dumps({'path': 'online inc', 'params': P,
                          'ms_per_upload': round(t * 1e3, 4),
                          'GBps_algorithmic': round(12.0 * P / t / 1e9, 1),
                          'what': 'OnlineClientsAvgAggregator.inc, device '
                                  'upload, 12 B/param'}), flush=True)
    if 'fedopt' in which:
        n = 100
        init = OrderedDict(w=torch.zeros(P, device=dev))
        clients = [(1 + i, OrderedDict(w=torch.randn(P, device=dev,
                                                     generator=g)))
                   for i in range(n)]
        info = {'client_feedback': clients, 'recover_fun': None}
        c = cfg()
        c.fedopt = SimpleNamespace(optimizer={'type': 'Adam', 'lr': 0.01},
                                   annealing=False)
        opt = FedOptAggregator(config=c, model=ParamModel(init), device=dev)
        avg = ClientsAvgAggregator(model=ParamModel(init), device=dev,
                                   config=cfg())
        t_opt = timed(lambda: opt.aggregate(info))
        t_avg = timed(lambda: avg.aggregate(info))
        print(json.dumps({'path': 'fedopt adam', 'clients': n, 'params': P,
                          'ms_aggregate': round(t_opt * 1e3, 4),
                          'ms_fedavg_same_dicts': round(t_avg * 1e3, 4),
                          'ms_step': round((t_opt - t_avg) * 1e3, 4),
                          'GBps_algorithmic': round(4.0 * n * P / t_opt / 1e9,
                                                    1),
                          'what': 'FedOptAggregator.aggregate (Adam): '
                                  'FedAvg + fused optimizer step'}),
              flush=True)


if __name__ == '__main__':
    main()
