#!/usr/bin/env python3
"""cProfile of the host side of multi-Krum aggregate() at C4 (device
select path, 50 device dicts, ConvNet2-h2048): 300 calls, each after a
synchronize; the top functions by own time and by cumulative time.
FRESH=1: new client addresses every call.  tools only."""
import cProfile
import io
import os
import pstats
import sys
from collections import OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench_robust import CONVNET2_H2048  # noqa: E402
from profile_rule import M, cfg  # noqa: E402


def main():
    from federatedscope_amd.core.aggregators import KrumAggregator
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(7)
    init = OrderedDict((k, torch.randn(s, device=dev, generator=g))
                       for k, s in CONVNET2_H2048)
    n = 50
    NOFF = 64 if os.environ.get('FRESH') else 1
    pools = [[1e-2 * torch.randn(int(np.prod(s)) + 64 * NOFF, device=dev,
                                 generator=g) for k, s in CONVNET2_H2048]
             for _ in range(n)]
    sets = [[(1 + i, OrderedDict(
        (k, pools[i][j][64 * c:64 * c + int(np.prod(s))].view(s))
        for j, (k, s) in enumerate(CONVNET2_H2048))) for i in range(n)]
        for c in range(NOFF)]
    agg = KrumAggregator(model=M(init), device=dev,
                         config=cfg(f=10, agg_num=5))
    for it in range(50):
        agg.aggregate({'client_feedback': sets[it % NOFF],
                       'recover_fun': None})
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    for it in range(300):
        torch.cuda.synchronize()
        pr.enable()
        agg.aggregate({'client_feedback': sets[it % NOFF],
                       'recover_fun': None})
        pr.disable()
    torch.cuda.synchronize()
    for key in ('tottime', 'cumulative'):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(45)
        print(s.getvalue())


if __name__ == '__main__':
    main()
