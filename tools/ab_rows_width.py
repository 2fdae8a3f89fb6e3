#!/usr/bin/env python3
"""A/B of the row-set weighted-sum kernel's chunk width V
(fsagg_wsum_set_rows_width) on separately allocated client keys: C5
(200 x ConvNet2-h2048, 6.6M, 12 keys) and the ResNet-50 layout (100 x 23.5M,
161 keys), against the flat kernel over a slab of the same shape.
Interleaved, median of 15 event-timed calls per round, 4 rounds; every
width's result must be identical to the default's.  tools only."""
import json
import os
import statistics
import sys
from collections import OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def run(lib, ops, lay, keys, n, widths, dev):
    g = torch.Generator(device=dev).manual_seed(n)
    clients = [OrderedDict((k, torch.randn(s, device=dev, generator=g))
                           for k, s in keys) for _ in range(n)]
    ptrs = np.array([[c[k].data_ptr() for k in lay.keys] for c in clients],
                    dtype=np.int64)
    rs = ops.RowSet.from_pointers(lay, ptrs, dev, keepalive=clients)
    sizes = [1 + (37 * i) % 1000 for i in range(n)]
    w = torch.tensor([s / sum(sizes) for s in sizes], dtype=torch.float32,
                     device=dev)
    out = torch.empty(lay.numel, device=dev)
    slab = torch.randn((n, ops.round_up(lay.numel, 64)), device=dev,
                       generator=g)
    flat_rows = ops.RowTable.from_slab(slab, numel=lay.numel)
    fout = torch.empty(slab.shape[1], device=dev)
    legs = {}
    for v in widths:
        def f(v=v):
            prev = lib.fsagg_wsum_set_rows_width(v)
            try:
                ops.weighted_sum_rows(rs, w, out)
            finally:
                lib.fsagg_wsum_set_rows_width(prev)
        legs['rows_v%d' % v] = f
    legs['flat'] = lambda: ops.weighted_sum(flat_rows, w, fout)
    ref = None
    same = {}
    for k, f in legs.items():
        if k == 'flat':
            continue
        f()
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        same[k] = bool(torch.equal(out, ref))
    res = {k: [] for k in legs}
    for rnd in range(4):
        order = list(legs) if rnd % 2 == 0 else list(legs)[::-1]
        for k in order:
            f = legs[k]
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            ts = []
            for _ in range(15):
                a, b = torch.cuda.Event(True), torch.cuda.Event(True)
                a.record()
                f()
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b))
            res[k].append(statistics.median(ts))
    med = {k: round(statistics.median(v), 4) for k, v in res.items()}
    return {'n': n, 'keys': len(keys), 'params': lay.numel, 'ms': med,
            'identical': same}


def main():
    from federatedscope_amd import _lib as L
    from federatedscope_amd import ops
    from federatedscope_amd.layout import BucketLayout
    from bench_robust import CONVNET2_H2048
    lib = L.load()
    dev = torch.device('cuda', 0)
    widths = [int(x) for x in os.environ.get('WIDTHS', '0,4,8,16,24').split(',')]
    lay = BucketLayout(OrderedDict((k, torch.empty(s, device='meta'))
                                   for k, s in CONVNET2_H2048))
    print(json.dumps(dict(run(lib, ops, lay, CONVNET2_H2048, 200, widths,
                              dev), layout='C5 ConvNet2-h2048')), flush=True)
    torch.cuda.empty_cache()
    with open(os.path.join(ROOT, 'tools', 'resnet50_layout.json')) as f:
        keys = [(k, tuple(s)) for k, s in json.load(f)['keys']]
    lay = BucketLayout(OrderedDict((k, torch.empty(s, device='meta'))
                                   for k, s in keys))
    print(json.dumps(dict(run(lib, ops, lay, keys, 100, widths, dev),
                          layout='ResNet-50')), flush=True)


if __name__ == '__main__':
    main()
