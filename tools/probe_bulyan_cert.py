#!/usr/bin/env python3
"""Why the Bulyan set certificate declines on the drop-in's i.i.d. data:
the score intervals around the cut from the Gram path's per-pair bounds,
split into the Gram arithmetic part and D's fp32 formation part; then the
whole aggregate() per trial (median of 10) and the distance path it took
(certified, refined from the ambiguous clients' fp64 rows, or recomputed)."""
import statistics
import time
import os
import sys
from collections import OrderedDict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import torch  # noqa: E402
from bench_robust import CONVNET2_H2048  # noqa: E402
from profile_rule import M, cfg  # noqa: E402


def main():
    from federatedscope_amd.core.aggregators import BulyanAggregator
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(7)
    init = OrderedDict((k, torch.randn(s, device=dev, generator=g))
                       for k, s in CONVNET2_H2048)
    for trial in range(4):
        clients = [(1 + i, OrderedDict(
            (k, 1e-2 * torch.randn(s, device=dev, generator=g))
            for k, s in CONVNET2_H2048)) for i in range(50)]
        agg = BulyanAggregator(model=M(init), device=dev,
                               config=cfg(f=10, client_num=50))
        st = agg._stage_all(clients)
        D = agg._pairdist(st).cpu().numpy().astype(np.float64)
        B = agg.last_pair_bound
        nseg = len(st.layout.keys)
        form = (2 * nseg + 2) * 2.0 ** -24 * np.where(np.isfinite(D), D, 0)
        n, f = 50, 10
        k = n - f - 2
        m = n - 2 * f
        sc = np.sort(D, 1)[:, :k].sum(1)
        order = np.argsort(sc)
        for name, BB in (('full', B), ('gram only', B - form),
                         ('formation only', form)):
            lo = np.sort(np.maximum(D - BB, 0), 1)[:, :k].sum(1)
            hi = np.sort(D + BB, 1)[:, :k].sum(1)
            top, rest = order[:m], order[m:]
            gap = lo[rest].min() - hi[top].max()
            print('trial %d %-15s cut gap %+.3e (rel %+.2e) B/D med %.2e' % (
                trial, name, gap, gap / sc.mean(),
                np.median((BB / D)[np.isfinite(D) & (D > 0)])))
        info = {'client_feedback': clients, 'recover_fun': None}
        ts = []
        for _ in range(12):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            agg.aggregate(info)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print('  score spacing at cut rel %.2e' % (
            (sc[order[m]] - sc[order[m - 1]]) / sc.mean()),
            'aggregate %.3f ms' % (statistics.median(ts[2:]) * 1e3),
            'path', agg.last_pairdist_path, flush=True)


if __name__ == '__main__':
    main()
