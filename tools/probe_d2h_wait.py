#!/usr/bin/env python3
"""How long the host takes to see a small device result (the Gram chain's
[5][n][n] finish buffer, 50 KB at n = 50) after the GPU produced it: the
chain plus (a) a blocking .cpu(), (b) a non-blocking copy into pinned
memory and event.synchronize(), (c) the same with a spin on event.query(),
each timed per call (median of 200).  tools only."""
import os
import statistics
import sys
import time
from collections import OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench_robust import CONVNET2_H2048  # noqa: E402


def main():
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import _GRAM_TOL
    from federatedscope_amd.layout import BucketLayout
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(7)
    clients = [OrderedDict((k, 1e-2 * torch.randn(s, device=dev, generator=g))
                           for k, s in CONVNET2_H2048) for _ in range(50)]
    lay = BucketLayout(OrderedDict((k, v.cpu()) for k, v in
                                   clients[0].items()))
    ptrs = np.array([[c[k].data_ptr() for k in lay.keys] for c in clients],
                    dtype=np.int64)
    rs = ops.RowSet.from_pointers(lay, ptrs, dev, keepalive=clients)
    pinned = torch.empty((5, 50, 50), dtype=torch.int32, pin_memory=True)
    ev = torch.cuda.Event()

    def a():
        buf = ops.pairgram_rows_dist(rs, _GRAM_TOL)[0]
        return buf.cpu()

    def b():
        buf = ops.pairgram_rows_dist(rs, _GRAM_TOL)[0]
        pinned.copy_(buf, non_blocking=True)
        ev.record()
        ev.synchronize()
        return pinned

    def c():
        buf = ops.pairgram_rows_dist(rs, _GRAM_TOL)[0]
        pinned.copy_(buf, non_blocking=True)
        ev.record()
        while not ev.query():
            pass
        return pinned

    def chain_only():
        ops.pairgram_rows_dist(rs, _GRAM_TOL)
        torch.cuda.synchronize()

    for name, fn in (('chain + synchronize', chain_only), ('a .cpu()', a),
                     ('b pinned + event.synchronize', b),
                     ('c pinned + query spin', c)):
        for _ in range(20):
            fn()
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        print('%-32s %.1f us' % (name, statistics.median(ts) * 1e6),
              flush=True)


if __name__ == '__main__':
    main()
