#!/usr/bin/env python3
"""A/B of the order-statistic kernels: for 64 < n <= 255 the two-wave form
(csrc/orderstat_pair.h) against the one-wave register select, for
255 < n <= 512 the K-wave form (csrc/orderstat_group.h, "two_wave" in the
output) against the two-pass streaming kernel ("one_wave"), interleaved
call by call in one process (fsagg_orderstat_set_pair_min moves the
dispatch), on C5-style data (N(0,1), 10 % of clients x100) at a fixed
4·n·P ≈ 5.3 GB (C5 itself at n = 200).  One JSON line per (n, rule).

  bench_pair.py [n ...]      (default: 72 100 128 160 200 255)
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from federatedscope_amd import _lib as L, ops  # noqa: E402

C5_P = 6_603_904


def timed_pair(fns, reps=12, rounds=3):
    """Median event time per fn, the fns interleaved round by round after a
    50 ms warm-up of each."""
    import time
    for fn in fns:
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.05:
            fn()
            torch.cuda.synchronize()
    ts = [[] for _ in fns]
    for _ in range(rounds):
        for i, fn in enumerate(fns):
            for _ in range(reps):
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                fn()
                b.record()
                b.synchronize()
                ts[i].append(a.elapsed_time(b))
    return [statistics.median(t) for t in ts]


def main():
    args = sys.argv[1:]
    rules = ('median', 'trimmed_mean')
    if args and args[0] in rules:
        rules, args = (args[0], ), args[1:]
    ns = [int(x) for x in args] or [72, 100, 128, 160, 200, 255]
    lib = L.load()
    dev = torch.device('cuda', 0)
    for n in ns:
        P = C5_P if n == 200 else int(4 * 200 * C5_P / (4 * n)) // 64 * 64
        g = torch.Generator(device=dev).manual_seed(2)
        slab = torch.randn((n, P), device=dev, generator=g)
        idx = torch.randperm(n, generator=torch.Generator().manual_seed(2))
        slab[idx[:n // 10]] *= 100.0
        rows = ops.RowTable.from_slab(slab)
        base = torch.randn(P, device=dev, generator=g)
        out = torch.empty(P, device=dev)
        k = int(n * 0.2)
        for rule in rules:
            def run(thr, rule=rule):
                def fn():
                    lib.fsagg_orderstat_set_pair_min(thr)
                    # n > 255: the K-wave kernel (thr 65) against the
                    # two-pass streaming kernel (thr 256)
                    lib.fsagg_orderstat_set_group_max(512 if thr == 65
                                                      else 255)
                    if rule == 'median':
                        ops.coord_median(rows, out, base=base)
                    else:
                        ops.trimmed_mean(rows, k, out, base=base)
                return fn
            one, pair = timed_pair([run(256), run(65)])
            nbytes = 4.0 * n * P + 8.0 * P
            print(json.dumps({
                'rule': rule, 'n': n, 'P': P, 'k': k if rule != 'median'
                else 0, 'one_wave_ms': round(one, 4),
                'two_wave_ms': round(pair, 4),
                'ratio_two_over_one': round(pair / one, 4),
                'two_wave_hbm_frac': round(nbytes / pair / 1e6 / 8000.0, 4),
                'one_wave_hbm_frac': round(nbytes / one / 1e6 / 8000.0, 4)}),
                flush=True)
        lib.fsagg_orderstat_set_pair_min(-1)
        lib.fsagg_orderstat_set_group_max(-1)
        del slab, rows, base, out
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
