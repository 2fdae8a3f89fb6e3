#!/usr/bin/env python3
"""Order-statistic kernels at other (clients × coordinates) shapes of the
same byte count as C5 (N(0,1) with 10 % of clients ×100): how the time per
byte moves with n (register-array size, hence waves per SIMD).  GPU only.

usage: os_shape.py N1,N2,...   (total bytes fixed at 200 × 6,603,904 × 4)
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from federatedscope_amd import ops  # noqa: E402


def timed(fn, reps=7):
    ts = []
    for _ in range(reps + 1):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts[1:])


def main():
    dev = torch.device('cuda', 0)
    total = 200 * 6603904
    for n in [int(x) for x in sys.argv[1].split(',')]:
        P = total // n // 256 * 256
        g = torch.Generator(device=dev).manual_seed(2)
        slab = torch.randn((n, P), device=dev, generator=g)
        idx = torch.randperm(n, generator=torch.Generator().manual_seed(2))
        slab[idx[:n // 10]] *= 100.0
        rows = ops.RowTable.from_slab(slab)
        out = torch.empty(P, device=dev)
        k = int(n * 0.2)
        tm = timed(lambda: ops.coord_median(rows, out))
        tt = timed(lambda: ops.trimmed_mean(rows, k, out))
        gb = 4.0 * n * P / 1e9
        print(json.dumps({'n': n, 'P': P, 'GB': round(gb, 3),
                          'median_ms': round(tm, 4),
                          'median_TBps': round(gb / tm, 3),
                          'trimmed_ms': round(tt, 4),
                          'trimmed_TBps': round(gb / tt, 3)}), flush=True)
        del slab, rows, out
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
