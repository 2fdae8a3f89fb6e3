#!/usr/bin/env python3
"""A/B of the Gram chain's LDS stages (fsagg_pairgram_set_stages): 1 the
compact stages (the n client rows, three buffers where they fit: two
stages in flight) against 0 the round-5 full-tile stages (16·NT rows + the
centre's, one in flight), interleaved, on C4's layout (ConvNet2-h2048,
6.6M, separately allocated keys) for the given n (default 50 100): median
of 15 event-timed calls of the whole chain (fsagg_pairgram_rows_f32) per
round, 4 rounds; D64 must be identical bit for bit.  KNOB=fused: the fused
chain tail (fsagg_pairgram_set_fused 1) against the round-5 eight launches
(0) instead.  tools only."""
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
    knob = os.environ.get('KNOB', 'stages')
    # MODES=a,b: the two settings compared (default 1,0; reported as
    # compact_* = a and fulltile_* = b)
    ma, mb = [int(x) for x in os.environ.get('MODES', '1,0').split(',')]
    setk = (lib.fsagg_pairgram_set_fused if knob == 'fused'
            else lib.fsagg_pairgram_set_stages)
    dev = torch.device('cuda', 0)
    ns = [int(a) for a in sys.argv[1:]] or [50, 100]
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
        bufs = {}
        for mode in (ma, mb):
            setk(mode)
            bufs[mode] = ops.pairgram_rows_dist(rs, _GRAM_TOL)[0].cpu().numpy()
        same = bufs[ma].tobytes() == bufs[mb].tobytes()
        res = {ma: [], mb: []}
        for rnd in range(int(os.environ.get('ROUNDS', '4'))):
            for mode in ((ma, mb) if rnd % 2 == 0 else (mb, ma)):
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
        setk(-1)
        print(json.dumps({'n': n, 'knob': knob, 'modes': [ma, mb], 'compact_ms': [round(x, 4) for x in res[ma]],
                          'fulltile_ms': [round(x, 4) for x in res[mb]],
                          'compact_median': round(statistics.median(res[ma]),
                                                  4),
                          'fulltile_median': round(statistics.median(res[mb]),
                                                   4),
                          'identical': same}), flush=True)
        del clients, rs
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
