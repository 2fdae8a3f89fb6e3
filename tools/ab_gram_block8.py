#!/usr/bin/env python3
"""A/B of the Gram chain for n > 64 (fsagg_pairgram_rows_f32): the workgroup
setting B8 (env, fsagg_pairgram_set_block8: 1 the default — one workgroup
holding every tile up to 112 clients, 8-tile workgroups up to 128, 13 tiles
on 16 waves above; 2 four 8-tile workgroups per chunk above 128; 3 the
one-workgroup form up to 128) against the plane-line workgroups (0),
interleaved, on C4's layout (ConvNet2-h2048,
6.6M) for n = 100 and 200: median of 15 event-timed calls per round, 3
rounds; the two D within 1e-6 relative of each other.  tools only."""
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
from bench_robust import CONVNET2_H2048  # noqa: E402


def main():
    from federatedscope_amd import _lib as L
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import _GRAM_TOL
    from federatedscope_amd.layout import BucketLayout
    lib = L.load()
    dev = torch.device('cuda', 0)
    ns = [int(a) for a in sys.argv[1:]] or [100, 200]
    for n in ns:
        g = torch.Generator(device=dev).manual_seed(n)
        clients = [OrderedDict((k, 1e-2 * torch.randn(s, device=dev,
                                                      generator=g))
                               for k, s in CONVNET2_H2048) for _ in range(n)]
        lay = BucketLayout(OrderedDict((k, v.cpu()) for k, v in
                                       clients[0].items()))
        ptrs = np.array([[c[k].data_ptr() for k in lay.keys]
                         for c in clients], dtype=np.int64)
        rs = ops.RowSet.from_pointers(lay, ptrs, dev, keepalive=clients)
        Ds = {}
        b8 = int(os.environ.get('B8', '1'))
        for on in (b8, 0):
            lib.fsagg_pairgram_set_block8(on)
            Ds[on] = ops.pairgram_rows_dist(rs, _GRAM_TOL)[4].cpu().numpy()
        off = ~np.eye(n, dtype=bool)
        rel = float(np.max(np.abs(Ds[b8][off] - Ds[0][off]) / Ds[0][off]))
        res = {b8: [], 0: []}
        for rnd in range(3):
            for on in ((b8, 0) if rnd % 2 == 0 else (0, b8)):
                lib.fsagg_pairgram_set_block8(on)
                for _ in range(5):
                    ops.pairgram_rows_dist(rs, _GRAM_TOL)
                torch.cuda.synchronize()
                ts = []
                e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
                for _ in range(15):
                    e0.record()
                    ops.pairgram_rows_dist(rs, _GRAM_TOL)
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1))
                res[on].append(statistics.median(ts))
        lib.fsagg_pairgram_set_block8(-1)
        print(json.dumps({'n': n, 'block8_ms': [round(x, 4) for x in res[b8]],
                          'lines_ms': [round(x, 4) for x in res[0]],
                          'block8_median': round(statistics.median(res[b8]), 4),
                          'lines_median': round(statistics.median(res[0]), 4),
                          'max_rel_diff_D64': rel}), flush=True)
        del clients, rs
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
