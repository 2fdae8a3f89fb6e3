#!/usr/bin/env python3
"""Order statistics for n <= 64 (the register sort kernel): coordinate median
and trimmed mean over n rows of 6.6M fp32 (Bulyan's 30 selected clients at
C4, and n = 50 / 64), timed with HIP events; checked against a torch sort of
sampled columns.  GPU only.  One JSON line per case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))

import torch  # noqa: E402
from bench_robust import timed  # noqa: E402


def main():
    from federatedscope_amd import ops
    dev = torch.device('cuda', 0)
    P = 6_603_904
    g = torch.Generator(device=dev).manual_seed(5)
    for n, k in ((30, 10), (50, 10), (64, 12)):
        X = torch.randn((n, P), device=dev, generator=g)
        rows = ops.RowTable.from_slab(X)
        out = torch.empty(P, device=dev)
        cols = torch.randint(0, P, (4096, ), device=dev, generator=g)
        S = torch.sort(X[:, cols].double(), dim=0)[0]
        for mode in ('median', 'trimmed'):
            if mode == 'median':
                fn = lambda: ops.coord_median(rows, out)  # noqa: E731
                want = ((S[(n - 1) // 2] + S[n // 2]) / 2).float()
            else:
                fn = lambda: ops.trimmed_mean(rows, k, out)  # noqa: E731
                want = (S[k:n - k].sum(0) / (n - 2 * k)).float()
            ms = timed(fn)
            err = (out[cols] - want).abs().max().item()
            print(json.dumps({
                'mode': mode, 'n': n, 'k': k if mode == 'trimmed' else 0,
                'P': P, 'ms_median': ms[0], 'ms_min': ms[1],
                'GBps': 4 * n * P / ms[0] / 1e6,
                'max_abs_err_sampled': err}), flush=True)
        del X, rows


if __name__ == '__main__':
    main()
