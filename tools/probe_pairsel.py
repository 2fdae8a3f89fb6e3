#!/usr/bin/env python3
"""Time fsagg_pairsel_* (the ambiguous clients' fp64 rows of Krum's D) at
the drop-in's shape (50 clients × CONVNET2_H2048) for 1..32 selected rows:
kernels alone (events) and the engine's whole refinement step."""
import os
import statistics
import sys
import time
from collections import OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import torch  # noqa: E402
from bench_robust import CONVNET2_H2048  # noqa: E402


def main():
    from federatedscope_amd import ops
    from federatedscope_amd.layout import BucketLayout
    import numpy as np
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(7)
    clients = [OrderedDict((k, 1e-2 * torch.randn(s, device=dev, generator=g))
                           for k, s in CONVNET2_H2048) for _ in range(50)]
    lay = BucketLayout(OrderedDict((k, v.cpu()) for k, v in
                                   clients[0].items()))
    ptrs = np.array([[c[k].data_ptr() for k in lay.keys] for c in clients],
                    dtype=np.int64)
    rs = ops.RowSet.from_pointers(lay, ptrs, dev, keepalive=clients)
    from federatedscope_amd import _lib as L
    for unit in (4096, 2048, 1024, 512):
        L.FSAGG_PAIRSEL_CHUNK = unit
        for nsel in (1, 2, 4, 8):
            sel = torch.arange(0, 50, 50 // nsel, dtype=torch.int32,
                               device=dev)[:nsel].contiguous()
            for _ in range(3):
                ops.pairsel_rows_segsq(rs, sel)
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ts = []
            for _ in range(20):
                ev[0].record()
                ops.pairsel_rows_segsq(rs, sel)
                ev[1].record()
                ev[1].synchronize()
                ts.append(ev[0].elapsed_time(ev[1]))
            print('chunk %4d nsel %2d: %.3f ms (events, segsq launch pair)' % (
                unit, nsel, statistics.median(ts)), flush=True)
    L.FSAGG_PAIRSEL_CHUNK = 2048
    for nsel in (1, 2, 4, 8, 16, 32):
        sel = torch.arange(0, 50, 50 // nsel if nsel <= 50 else 1,
                           dtype=torch.int32, device=dev)[:nsel].contiguous()
        for _ in range(3):
            ops.pairsel_finish(ops.pairsel_rows_segsq(rs, sel), sel)
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            t0 = time.perf_counter()
            ops.pairsel_finish(ops.pairsel_rows_segsq(rs, sel), sel).cpu()
            ts.append(time.perf_counter() - t0)
        print('nsel %2d: %.3f ms (host-timed, incl. D copy)' % (
            nsel, statistics.median(ts) * 1e3), flush=True)


if __name__ == '__main__':
    main()
