#!/usr/bin/env python3
"""Host timeline of one multi-Krum aggregate() at C4 on the device-select
path (50 device dicts, ConvNet2-h2048, f = 10, 5 selected): the time from
the call's start at which each step returns (median µs over 200 calls, each
after a synchronize), taken by wrapping the steps KrumAggregator._krum_device
runs — staging, the Gram chain's launch, the base table, the selection's
launch, the average's launch, the host's wait — plus the GPU's own time
from the first kernel of the call to its last (HIP events on the stream).
FRESH=1: new client addresses every call.  tools only."""
import os
import statistics
import sys
import time
from collections import OrderedDict, defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench_robust import CONVNET2_H2048  # noqa: E402
from profile_rule import M, cfg  # noqa: E402


def main():
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators import KrumAggregator
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(7)
    init = OrderedDict((k, torch.randn(s, device=dev, generator=g))
                       for k, s in CONVNET2_H2048)
    fresh = bool(os.environ.get('FRESH'))
    n = int(os.environ.get('N', '50'))
    NOFF = 440 if fresh else 1
    pools = [[1e-2 * torch.randn(int(np.prod(s)) + 64 * NOFF, device=dev,
                                 generator=g) for k, s in CONVNET2_H2048]
             for _ in range(n)]
    sets = [[(1 + i, OrderedDict(
        (k, pools[i][j][64 * c:64 * c + int(np.prod(s))].view(s))
        for j, (k, s) in enumerate(CONVNET2_H2048))) for i in range(n)]
        for c in range(NOFF)]
    nxt = [0]

    def next_models():
        nxt[0] = (nxt[0] + 1) % NOFF
        return sets[nxt[0]]
    agg = KrumAggregator(model=M(init), device=dev,
                         config=cfg(f=10, agg_num=5))
    marks = defaultdict(list)
    t0 = [0.0]
    on = [False, 0]

    def wrap(obj, name, label):
        fn = getattr(obj, name)

        def w(*a, **k):
            r = fn(*a, **k)
            if on[0] and len(marks[label]) < on[1]:
                marks[label].append((time.perf_counter() - t0[0]) * 1e6)
            return r
        setattr(obj, name, w)
    wrap(agg, '_stage_all', '1 staged')
    wrap(ops, '_require_all', '2a0 require_all')
    wrap(ops._GRAPHS, 'lookup', '2a1 graph lookup')
    wrap(torch.cuda.CUDAGraph, 'replay', '2a3 replayed')
    wrap(torch.cuda.Event, 'synchronize', '2a2 event sync (1st)')
    wrap(agg, '_pairdist', '2 gram launched')
    wrap(agg, '_base', '3 base table')
    wrap(ops, 'krum_select', '4 select launched')
    wrap(ops, 'weighted_sum_rows_devtab', '5 average launched')
    gpu = []
    for it in range(260):
        models = next_models()
        torch.cuda.synchronize()
        on[0] = it >= 60
        on[1] = it - 59
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        t0[0] = time.perf_counter()
        e0.record()
        agg.aggregate({'client_feedback': models, 'recover_fun': None})
        t1 = (time.perf_counter() - t0[0]) * 1e6
        e1.record()
        torch.cuda.synchronize()
        if on[0]:
            marks['6 returned'].append(t1)
            gpu.append(e0.elapsed_time(e1) * 1e3)
    for k in sorted(marks):
        print('%-20s %7.1f us' % (k, statistics.median(marks[k])))
    print('events first..last  %7.1f us (GPU span incl. host gaps)'
          % statistics.median(gpu))
    print('path', agg.last_pairdist_path, 'selection', agg.last_selection)


if __name__ == '__main__':
    main()
