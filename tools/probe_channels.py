#!/usr/bin/env python3
"""The channel hypothesis of the layout-B gap (verdict
item 3): the row-set FedAvg kernel over 100 clients x the ResNet-50 layout
(161 keys), with each client's keys of >= 1 MiB placed
  sep      as torch allocates separate tensors (clones: 2 MiB-aligned blocks)
  aligned  in one buffer per key, client i at i x round_up(bytes, 2 MiB)
           (the same alignment, chosen by us)
  stagger  the same buffer, client i shifted by a different multiple of
           4 KiB within the 2 MiB window
(smaller keys: clones in every leg), against the flat kernel over the slab
rows.  Interleaved, median of rounds of back-to-back calls; every leg's
result bit-identical to the flat kernel's.  tools only.

    python tools/probe_channels.py [--rounds 5] [--calls 10]
"""
import argparse
import json
import os
import statistics
import sys
import time
from collections import OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

MIB2 = 2 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--clients', type=int, default=100)
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--calls', type=int, default=10)
    args = ap.parse_args()
    from federatedscope_amd import ops
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
    tot = float(sum(sizes))
    w = torch.tensor([s / tot for s in sizes], dtype=torch.float32,
                     device=dev)

    def view(i, k):
        o = lay.offsets[k]
        return slab[i, o:o + lay.numels[k]]

    keep = []

    def placed(mode):
        """[n][nseg] pointers of the clients' keys placed by ``mode``."""
        ptrs = np.zeros((n, len(lay.keys)), dtype=np.int64)
        for s, k in enumerate(lay.keys):
            m = lay.numels[k]
            if mode == 'sep' or 4 * m < (1 << 20):
                for i in range(n):
                    t = view(i, k).clone()
                    keep.append(t)
                    ptrs[i, s] = t.data_ptr()
                continue
            stride = ops.round_up(4 * m, MIB2)
            buf = torch.empty((n * stride + MIB2) // 4, dtype=torch.float32,
                              device=dev)
            keep.append(buf)
            for i in range(n):
                shift = 0 if mode == 'aligned' else \
                    ((i * 2053) % 512) * 4096
                o = (i * stride + shift) // 4
                buf[o:o + m].copy_(view(i, k))
                ptrs[i, s] = buf.data_ptr() + 4 * o
        return ops.RowSet.from_pointers(lay, ptrs, dev, keepalive=tuple(keep))

    sets = {m: placed(m) for m in ('sep', 'aligned', 'stagger')}
    outs = {m: torch.empty(ld, dtype=torch.float32, device=dev) for m in sets}
    flat = torch.empty(ld, dtype=torch.float32, device=dev)
    rows = ops.RowTable.from_slab(slab, numel=ld)
    legs = {'rows_' + m: (lambda m=m: ops.weighted_sum_rows(sets[m], w,
                                                            outs[m]))
            for m in sets}
    legs['flat'] = lambda: ops.weighted_sum(rows, w, flat)
    for fn in legs.values():
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    exact = {m: all(torch.equal(outs[m][lay.offsets[k]:lay.offsets[k] +
                                        lay.numels[k]],
                                flat[lay.offsets[k]:lay.offsets[k] +
                                     lay.numels[k]]) for k in lay.keys)
             for m in sets}
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
    rec = {'keys': len(keys), 'params': P, 'clients': n,
           'bit_exact': exact}
    rec.update({k + '_ms': round(v, 4) for k, v in med.items()})
    rec.update({k + '_over_flat': round(v / med['flat'], 4)
                for k, v in med.items() if k != 'flat'})
    print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
