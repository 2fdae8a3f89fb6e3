#!/usr/bin/env python3
"""Where the multi-key FedAvg time goes (configs[2] layout B: the ResNet-50
layout, 161 keys, 100 clients).

Times, interleaved (median of rounds of back-to-back calls):
  agg_views   ClientsAvgAggregator.aggregate() on dicts whose keys are views
              of one slab row per client (bench.py's plugin_surface_layout_b)
  agg_sep     the same on separately allocated key tensors (a deserialised
              or per-module state_dict)
  rows_views  ops.weighted_sum_rows on the views' row set (kernel + launch)
  rows_sep    the same on the separate tensors' row set
  flat        ops.weighted_sum over the slab rows (the flat kernel)
Run under rocprofv3 --kernel-trace --stats for the kernels' own durations.
--rows-widths 0,24,8 adds rows_sep_V / agg_sep_V legs at a fixed row-set
chunk width (fsagg_wsum_set_rows_width).

    python tools/probe_layout_b.py [--rounds 5] [--calls 10] [--only rows_sep]
"""
import argparse
import json
import os
import statistics
import sys
import time
from collections import OrderedDict
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--clients', type=int, default=100)
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--calls', type=int, default=10)
    ap.add_argument('--only', default=None,
                    help='comma-separated legs to run (for per-leg counter '
                         'passes), e.g. rows_sep')
    ap.add_argument('--rows-widths', default=None,
                    help='comma-separated row-set chunk widths V to time as '
                         'extra legs rows_sep_V / agg_sep_V '
                         '(fsagg_wsum_set_rows_width; 0 = the rule)')
    ap.add_argument('--no-fill', action='store_true',
                    help='allocate the separate tensors without copying the '
                         'values in (16100 copy kernels are slow under a '
                         'counter pass; the timings do not depend on values)')
    args = ap.parse_args()
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.layout import BucketLayout
    dev = torch.device('cuda', 0)
    with open(os.path.join(ROOT, 'tools', 'resnet50_layout.json')) as f:
        keys = [(k, tuple(s)) for k, s in json.load(f)['keys']]
    lay = BucketLayout(OrderedDict((k, torch.empty(s, device='meta'))
                                   for k, s in keys))
    n, P = args.clients, lay.numel
    ld = ops.round_up(P, 64)
    slab = torch.empty((n, ld), dtype=torch.float32, device=dev)
    ops.fill_uniform(slab, ld, seed=7)
    sizes = [1 + (37 * i) % 1000 for i in range(n)]
    views = [(sizes[i], OrderedDict(
        (k, slab[i, lay.offsets[k]:lay.offsets[k] + lay.numels[k]].view(
            lay.shapes[k])) for k in lay.keys)) for i in range(n)]
    sep = [(s, OrderedDict((k, torch.empty_like(v) if args.no_fill
                            else v.clone()) for k, v in d.items()))
           for s, d in views]
    cfg = SimpleNamespace(federate=SimpleNamespace(ignore_weight=False,
                                                   use_ss=False))
    agg = ClientsAvgAggregator(device=dev, config=cfg)
    tot = float(sum(sizes))
    w = torch.tensor([s / tot for s in sizes], dtype=torch.float32,
                     device=dev)

    def rowset(cl):
        ptrs = np.array([[d[k].data_ptr() for k in lay.keys] for _, d in cl],
                        dtype=np.int64)
        return ops.RowSet.from_pointers(lay, ptrs, dev, keepalive=cl)

    rs_v, rs_s = rowset(views), rowset(sep)
    out = torch.empty(ld, dtype=torch.float32, device=dev)
    flat = torch.empty(ld, dtype=torch.float32, device=dev)
    rows = ops.RowTable.from_slab(slab, numel=ld)
    legs = {
        'agg_views': lambda: agg.aggregate({'client_feedback': views}),
        'agg_sep': lambda: agg.aggregate({'client_feedback': sep}),
        'rows_views': lambda: ops.weighted_sum_rows(rs_v, w, out),
        'rows_sep': lambda: ops.weighted_sum_rows(rs_s, w, out),
        'flat': lambda: ops.weighted_sum(rows, w, flat),
    }
    if args.rows_widths:
        from federatedscope_amd import _lib as L
        lib = L.load()

        def at(v, fn):
            def run():
                prev = lib.fsagg_wsum_set_rows_width(v)
                try:
                    return fn()
                finally:
                    lib.fsagg_wsum_set_rows_width(prev)
            return run
        for v in [int(x) for x in args.rows_widths.split(',')]:
            legs['rows_sep_%d' % v] = at(v, legs['rows_sep'])
            legs['agg_sep_%d' % v] = at(v, legs['agg_sep'])
    if args.only:
        keep = args.only.split(',') + ['flat']
        legs = {k: v for k, v in legs.items() if k in keep}
    for fn in legs.values():
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    ts = {k: [] for k in legs}
    for _ in range(args.rounds):
        for k, fn in legs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.calls):
                fn()
            torch.cuda.synchronize()
            ts[k].append((time.perf_counter() - t0) / args.calls * 1e3)
    med = {k: statistics.median(v) for k, v in ts.items()}
    rec = {'keys': len(keys), 'params': P, 'clients': n}
    rec.update({k + '_ms': round(v, 4) for k, v in med.items()})
    rec.update({k + '_over_flat': round(v / med['flat'], 4)
                for k, v in med.items() if k != 'flat'})
    print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
