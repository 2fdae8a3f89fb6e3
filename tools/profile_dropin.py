#!/usr/bin/env python3
"""cProfile of one drop-in aggregate() on device-resident ConvNet2 dicts
(host-side overhead hunting; GPU only)."""
import cProfile
import os
import pstats
import sys
from collections import OrderedDict
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))

import torch  # noqa: E402
from bench_robust import CONVNET2_H2048  # noqa: E402


def main():
    from federatedscope_amd.core.aggregators import (ClientsAvgAggregator,
                                                     MedianAggregator)
    rule = sys.argv[1] if len(sys.argv) > 1 else 'fedavg'
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(7)
    init = OrderedDict((k, torch.randn(s, device=dev, generator=g))
                       for k, s in CONVNET2_H2048)

    class M(torch.nn.Module):
        def state_dict(self, *a, **kw):
            return OrderedDict((k, v.clone()) for k, v in init.items())

    cfg = SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=1000, sample_client_rate=1.0),
        aggregator=SimpleNamespace(byzantine_node_num=0, BFT_args=None))
    agg = (ClientsAvgAggregator if rule == 'fedavg' else MedianAggregator)(
        model=M(), device=dev, config=cfg)
    fb = [(1 + i, OrderedDict((k, torch.randn(s, device=dev, generator=g))
                              for k, s in CONVNET2_H2048))
          for i in range(200)]
    info = {'client_feedback': fb, 'recover_fun': None}
    agg.aggregate(info)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        agg.aggregate(info)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats('tottime').print_stats(25)


if __name__ == '__main__':
    main()
