#!/usr/bin/env python3
"""Host timeline of one multi-Krum aggregate() at C4 (50 device dicts,
ConvNet2-h2048, f = 10, 5 selected): perf_counter marks between the phases
of KrumAggregator._krum_device (median µs from the call's start over 200
calls, each call after a synchronize).  tools only."""
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
    from federatedscope_amd.core.aggregators import KrumAggregator
    from federatedscope_amd.core.aggregators._engine import fedavg_weights
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(7)
    init = OrderedDict((k, torch.randn(s, device=dev, generator=g))
                       for k, s in CONVNET2_H2048)
    fresh = bool(os.environ.get('FRESH'))
    if fresh:
        # fresh uploads: every call's clients at new addresses (views at a
        # new offset into per-key pools), as a server round's new tensors
        import numpy as np
        NOFF = 440
        pools = [[1e-2 * torch.randn(int(np.prod(s)) + 64 * NOFF, device=dev,
                                     generator=g) for k, s in CONVNET2_H2048]
                 for _ in range(50)]
        sets = [[(1 + i, OrderedDict(
            (k, pools[i][j][64 * c:64 * c + int(np.prod(s))].view(s))
            for j, (k, s) in enumerate(CONVNET2_H2048))) for i in range(50)]
            for c in range(NOFF)]
    models = [(1 + i, OrderedDict(
        (k, 1e-2 * torch.randn(s, device=dev, generator=g))
        for k, s in CONVNET2_H2048)) for i in range(50)]
    nxt = [0]

    def next_models():
        if not fresh:
            return models
        nxt[0] += 1
        return sets[nxt[0] - 1]
    agg = KrumAggregator(model=M(init), device=dev,
                         config=cfg(f=10, agg_num=5))
    marks = defaultdict(list)

    def one():
        models = next_models()
        t0 = time.perf_counter()
        m = lambda k: marks[k].append((time.perf_counter() - t0) * 1e6)
        st = agg._stage_all(models)
        m('1 staged')
        D = agg._pairdist(st)
        m('2 gram launched')
        base = agg._base(st.layout, agg.model.state_dict(), as_float=True)
        m('3 base table')
        Dh = D.cpu()
        m('4 D on host')
        _, _, order = agg._certified_order(st, Dh, 10, 5, ordered=True)
        m('5 certified')
        sel = [int(i) for i in order[:5]]
        sizes = [models[i][0] for i in sel]
        weights = fedavg_weights(sizes, False)
        sub = st.subset(sel)
        m('6 subset')
        out = agg._run_pieces(sub, lambda rs, o, lo, hi: ops.weighted_sum_rows(
            rs, weights, o, base=base, lo=lo, hi=hi))
        m('7 wsum launched')
        res = agg._emit(st.layout, out, list(models[0][1].keys()),
                        models[0][1][next(iter(models[0][1]))].device)
        m('8 emitted')
        torch.cuda.synchronize()
        m('9 synchronized')
        return res

    for _ in range(30):
        one()
    marks.clear()
    for _ in range(200):
        torch.cuda.synchronize()
        one()
    ts = []
    for _ in range(200):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        agg.aggregate({'client_feedback': next_models(),
                       'recover_fun': None})
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    for k in sorted(marks):
        print('%-18s %7.1f us' % (k, statistics.median(marks[k])))
    print('aggregate() synchronised %.1f us' % statistics.median(ts))


if __name__ == '__main__':
    main()
