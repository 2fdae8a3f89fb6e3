#!/usr/bin/env python3
"""Host timeline of the median drop-in at C5 (200 device dicts,
ConvNet2-h2048, 12 separately allocated keys): perf_counter marks at the
return of each step of MedianAggregator.aggregate, median µs over 100 calls
(each after a synchronize), and the aggregate() wall time against the
kernel's own event time.  tools only."""
import os
import statistics
import sys
import time
from collections import OrderedDict, defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import torch  # noqa: E402
from bench_robust import CONVNET2_H2048  # noqa: E402
from profile_rule import M, cfg  # noqa: E402


def main():
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators import MedianAggregator
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(7)
    init = OrderedDict((k, torch.randn(s, device=dev, generator=g))
                       for k, s in CONVNET2_H2048)
    models = [(1 + i, OrderedDict((k, torch.randn(s, device=dev, generator=g))
                                  for k, s in CONVNET2_H2048))
              for i in range(200)]
    agg = MedianAggregator(model=M(init), device=dev, config=cfg(f=10))
    marks = defaultdict(list)
    t0 = [0.0]
    on = [False]

    def wrap(obj, name, label):
        fn = getattr(obj, name)

        def w(*a, **k):
            r = fn(*a, **k)
            if on[0]:
                marks[label].append((time.perf_counter() - t0[0]) * 1e6)
            return r
        setattr(obj, name, w)
    wrap(agg, '_stage_all', '1 staged')
    wrap(agg, '_base', '2 base')
    wrap(ops, 'coord_median_rows', '3 kernel launched')
    wrap(agg, '_emit', '4 emitted')
    kern = []
    for it in range(130):
        torch.cuda.synchronize()
        on[0] = it >= 30
        t0[0] = time.perf_counter()
        a = torch.cuda.Event(True)
        b = torch.cuda.Event(True)
        a.record()
        agg.aggregate({'client_feedback': models, 'recover_fun': None})
        b.record()
        torch.cuda.synchronize()
        if on[0]:
            marks['5 synchronised'].append((time.perf_counter() - t0[0]) * 1e6)
            kern.append(a.elapsed_time(b) * 1e3)
    for k in sorted(marks):
        print('%-20s %7.1f us' % (k, statistics.median(marks[k])))
    print('events around the call %7.1f us' % statistics.median(kern))


if __name__ == '__main__':
    main()
