#!/usr/bin/env python3
"""cProfile of one drop-in rule's aggregate() on device-resident C4/C5-shape
dicts (tools/bench_robust.py dropin's data): the synchronised call time,
the host-only time (no synchronize inside the loop), and the top host
functions by total time.  GPU only.

  profile_rule.py krum|bulyan|fedavg|median|trimmed|layout_b
"""
import cProfile
import io
import os
import pstats
import statistics
import sys
import time
from collections import OrderedDict
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))

import torch  # noqa: E402
from bench_robust import CONVNET2_H2048  # noqa: E402


def cfg(f=0, agg_num=1, ratio=0.2, client_num=1000):
    bft = SimpleNamespace(krum_agg_num=agg_num,
                          trimmedmean_excluded_ratio=ratio,
                          normbounding_norm_bound=5.0)
    return SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=client_num,
                                 sample_client_rate=1.0),
        aggregator=SimpleNamespace(byzantine_node_num=f, BFT_args=bft),
        asyn=SimpleNamespace(staleness_discount_factor=1.0))


class M(torch.nn.Module):
    def __init__(self, sd):
        super().__init__()
        self._sd = sd

    def state_dict(self, *a, **kw):
        return self._sd


def main():
    import json
    from federatedscope_amd.core.aggregators import (
        BulyanAggregator, ClientsAvgAggregator, KrumAggregator,
        MedianAggregator, TrimmedmeanAggregator)
    rule = sys.argv[1]
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(7)
    keys = CONVNET2_H2048
    if rule == 'layout_b':
        with open(os.path.join(ROOT, 'tools', 'resnet50_layout.json')) as f:
            keys = [(k, tuple(s)) for k, s in json.load(f)['keys']]
    init = OrderedDict((k, torch.randn(s, device=dev, generator=g))
                       for k, s in keys)
    n = {'krum': 50, 'bulyan': 50, 'layout_b': 100}.get(rule, 200)
    clients = [(int(1 + i), OrderedDict(
        (k, 1e-2 * torch.randn(s, device=dev, generator=g))
        for k, s in keys)) for i in range(n)]
    agg = {
        'krum': lambda: KrumAggregator(model=M(init), device=dev,
                                       config=cfg(f=10, agg_num=5)),
        'bulyan': lambda: BulyanAggregator(model=M(init), device=dev,
                                           config=cfg(f=10, client_num=50)),
        'fedavg': lambda: ClientsAvgAggregator(model=M(init), device=dev,
                                               config=cfg()),
        'layout_b': lambda: ClientsAvgAggregator(model=M(init), device=dev,
                                                 config=cfg()),
        'median': lambda: MedianAggregator(model=M(init), device=dev,
                                           config=cfg()),
        'trimmed': lambda: TrimmedmeanAggregator(model=M(init), device=dev,
                                                 config=cfg()),
    }[rule]()
    info = {'client_feedback': clients, 'recover_fun': None}
    for _ in range(30):
        agg.aggregate(info)
    torch.cuda.synchronize()
    sync, host = [], []
    for _ in range(40):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        agg.aggregate(info)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e6)
        sync.append((t2 - t0) * 1e6)
    print('%s: synchronised %.1f us, host part %.1f us (medians), path %s' %
          (rule, statistics.median(sync), statistics.median(host),
           getattr(agg, 'last_pairdist_path', None)))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(100):
        agg.aggregate(info)
        torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats('tottime').print_stats(30)
    print(s.getvalue())


if __name__ == '__main__':
    main()
