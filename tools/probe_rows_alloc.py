#!/usr/bin/env python3
"""Probe (tools only): the FedAvg kernels at 100 x 25M on the same values laid
out two ways — one slab (rows 100 MB apart, not 2 MiB aligned) and 100
separate allocations (each row 2 MiB aligned, as the clients' own tensors
are) — through the flat kernel (fsagg_weighted_sum_f32) and the row-set
kernel (fsagg_weighted_sum_rows_f32).  Median of 10 event-timed calls.
GPU only."""
import json
import os
import statistics
import sys
from collections import OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from federatedscope_amd import ops  # noqa: E402
from federatedscope_amd.layout import BucketLayout  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    n, P = 100, 25_000_000
    dev = torch.device('cuda', 0)
    w = [1.0 / n] * n
    slab = torch.empty((n, P), device=dev)
    ops.fill_uniform(slab, P, seed=1)
    sep = [slab[i].clone() for i in range(n)]
    out = torch.empty(P, device=dev)
    lay = BucketLayout(OrderedDict(w=torch.empty(P)))
    res = {}
    rs_slab = ops.RowSet.from_pointers(
        lay, [[slab[i].data_ptr()] for i in range(n)], dev, keepalive=(slab,))
    rs_sep = ops.RowSet.from_pointers(
        lay, [[t.data_ptr()] for t in sep], dev, keepalive=(sep,))
    runs = {
        'flat_slab': lambda: ops.weighted_sum(
            ops.RowTable.from_slab(slab), w, out),
        'flat_separate': lambda: ops.weighted_sum(
            ops.RowTable([t.data_ptr() for t in sep], P, dev, keepalive=sep),
            w, out),
        'rows_slab': lambda: ops.weighted_sum_rows(rs_slab, w, out),
        'rows_separate': lambda: ops.weighted_sum_rows(rs_sep, w, out),
    }
    # FSAGG_PROBE_ORDER=reverse runs them last to first (the clocks drift
    # over a run: the order must not decide the comparison)
    order = list(runs)
    mode = os.environ.get('FSAGG_PROBE_ORDER')
    if mode == 'reverse':
        order.reverse()
    if mode == 'interleave':
        # one call of each case in turn, 12 rounds: every case sees the
        # same drift
        ts = {k: [] for k in order}
        for _ in range(12):
            for k in order:
                ts[k].append(timed(runs[k], reps=1))
        for k in order:
            res[k] = statistics.median(ts[k][2:])
    else:
        for k in order:
            res[k] = timed(runs[k])
    res['row_addr_mod_2MiB'] = sorted({t.data_ptr() % (1 << 21)
                                       for t in sep})[:4]
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v)
                      for k, v in res.items()}), flush=True)


if __name__ == '__main__':
    main()
