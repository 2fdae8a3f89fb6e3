#!/usr/bin/env python3
"""Probe: the Gram Krum path's time against the data and the memory
layout at the C4 shape (50 clients, ConvNet2-h2048 keys): a slab with the
C4 mix (common base, Byzantine cluster) or i.i.d. N(0,1), read as per-key
views of the slab rows or as separately allocated key tensors.  GPU only."""
import json
import os
import sys
from collections import OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench_robust import layout, timed  # noqa: E402


def main():
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import _GRAM_TOL
    dev = torch.device('cuda', 0)
    lay = layout()
    P, n = lay.numel, 50
    g = torch.Generator(device=dev).manual_seed(1234)
    base = torch.randn(P, device=dev, generator=g)
    slab = torch.empty((n, P), device=dev)
    for kind in ('c4', ):
        for r in range(n):
            z = torch.randn(P, device=dev, generator=g)
            if kind == 'c4':
                slab[r] = (0.1 + 0.05 * z) if r % 5 == 0 else \
                    base + 0.01 * (1 + 0.05 * r) * z
            elif kind == 'iid':
                slab[r] = z
            elif kind == 'iid_scaled':
                slab[r] = 0.01 * z
            else:
                slab[r] = 0.0
        for form in ('views', 'separate', 'separate_skewed', 'views_aligned'):
            if form == 'separate_skewed':
                # separately allocated rows, each at a different offset mod
                # 2 MiB (i x 4 KiB + i x 256 B into an oversized buffer)
                ts = []
                for i in range(n):
                    row = []
                    for k in lay.keys:
                        m = lay.numels[k]
                        sk = (i * 1088) % 524288
                        buf = torch.empty(m + sk, device=dev)
                        buf[sk:] = slab[i, lay.offsets[k]:lay.offsets[k] + m]
                        row.append(buf[sk:])
                    ts.append(row)
                ptrs = [[t.data_ptr() for t in row] for row in ts]
                keep = (ts, )
            elif form == 'views_aligned':
                # one allocation, rows 2 MiB-aligned (stride a multiple of
                # 2 MiB)
                stride = (P + 524287) // 524288 * 524288
                big = torch.zeros((n, stride), device=dev)
                big[:, :P] = slab
                ptrs = [[big[i, lay.offsets[k]:].data_ptr() for k in
                         lay.keys] for i in range(n)]
                keep = (big, )
            elif form == 'views':
                ptrs = [[slab[i, lay.offsets[k]:].data_ptr() for k in
                         lay.keys] for i in range(n)]
                keep = (slab, )
            else:
                ts = [[slab[i, lay.offsets[k]:lay.offsets[k] +
                            lay.numels[k]].clone() for k in lay.keys]
                      for i in range(n)]
                ptrs = [[t.data_ptr() for t in row] for row in ts]
                keep = (ts, )
            fc1 = lay.keys.index('fc1.weight')
            offs = len({row[fc1] % (1 << 21) for row in ptrs})
            rs = ops.RowSet.from_pointers(lay, np.array(ptrs, dtype=np.int64),
                                          dev, keepalive=keep)

            def run():
                return ops.pairgram_rows_dist(rs, _GRAM_TOL)

            def valu():
                return ops.pairdist_finish(ops.pairdist_rows_segsq(rs))
            run()
            med, mn = timed(run)
            vmed, vmn = timed(valu)
            print(json.dumps({'lib': os.environ.get('FSAGG_LIB', 'product'),
                              'data': kind, 'form': form,
                              'gram_ms_median': med, 'gram_ms_min': mn,
                              'valu_ms_median': vmed,
                              'distinct_fc1_offsets_mod_2MiB': offs}),
                  flush=True)


if __name__ == '__main__':
    main()
