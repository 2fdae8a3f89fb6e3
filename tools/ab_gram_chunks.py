#!/usr/bin/env python3
"""A/B of a Gram chain knob — the main-pass chunk count
(fsagg_pairgram_set_chunks: $CHUNKS, default 1024,512,768) or, with
KNOB=desync, the main pass's start offset (fsagg_pairgram_set_desync:
$CHUNKS as its settings) — interleaved, on C4's layout
(ConvNet2-h2048, 6.6M, separately allocated keys) for the given n (default
50): median of 15 event-timed calls of the whole chain
(fsagg_pairgram_rows_f32) per round, 4 rounds; D64 within 1e-12 relative
(only the fp64 order of the chunk sums changes).  tools only."""
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
    setk = (lib.fsagg_pairgram_set_desync
            if os.environ.get('KNOB') == 'desync'
            else lib.fsagg_pairgram_set_chunks)
    dev = torch.device('cuda', 0)
    ns = [int(a) for a in sys.argv[1:]] or [50]
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
        modes = [int(x) for x in os.environ.get('CHUNKS',
                                                '1024,512,768').split(',')]
        d64 = {}
        for mode in modes:
            setk(mode)
            d64[mode] = ops.pairgram_rows_dist(rs, _GRAM_TOL)[4].cpu().numpy()
        off = ~np.eye(n, dtype=bool)
        rel = max(float(np.max(np.abs(d64[m][off] - d64[modes[0]][off]) /
                               d64[modes[0]][off])) for m in modes)
        res = {m: [] for m in modes}
        for rnd in range(4):
            for mode in (modes if rnd % 2 == 0 else modes[::-1]):
                setk(mode)
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
                res[mode].append(statistics.median(ts))
        setk(0)
        print(json.dumps({'n': n, 'knob': os.environ.get('KNOB', 'chunks'),
                          'chunks_ms': {
            str(m): [round(x, 4) for x in res[m]] for m in modes},
            'median_ms': {str(m): round(statistics.median(res[m]), 4)
                          for m in modes},
            'max_rel_diff_D64': rel}), flush=True)
        del clients, rs
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
