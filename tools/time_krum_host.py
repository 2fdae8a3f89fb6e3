#!/usr/bin/env python3
"""Host-side phases of KrumAggregator.distance_matrix on 50 device-resident
ConvNet2-h2048 dicts (C4 shape): each phase wrapped with perf_counter (no
device synchronisation inside), mean microseconds per call, against the
call's synchronised wall time and the GPU time of its kernels (events on
the launch stream).  GPU only."""
import functools
import json
import os
import sys
import time
from collections import OrderedDict, defaultdict
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))

import torch  # noqa: E402
from bench_robust import CONVNET2_H2048  # noqa: E402

ACC = defaultdict(float)
CNT = defaultdict(int)


def wrap(obj, name, label):
    f = getattr(obj, name)

    @functools.wraps(f)
    def g(*a, **kw):
        t0 = time.perf_counter()
        try:
            return f(*a, **kw)
        finally:
            ACC[label] += time.perf_counter() - t0
            CNT[label] += 1
    setattr(obj, name, g)


def main():
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators import KrumAggregator, _engine
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(7)
    cfg = SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=1000, sample_client_rate=1.0),
        aggregator=SimpleNamespace(byzantine_node_num=10,
                                   BFT_args=SimpleNamespace(krum_agg_num=1)))
    agg = KrumAggregator(device=dev, config=cfg)
    fb = [(1 + i, OrderedDict((k, torch.randn(s, device=dev, generator=g))
                              for k, s in CONVNET2_H2048))
          for i in range(50)]
    for _ in range(5):
        agg.distance_matrix(fb)
    torch.cuda.synchronize()
    wrap(_engine.DeviceEngine, '_stage_all', 'stage_all (key table, rows)')
    wrap(ops, 'pairgram_rows_dist', 'pairgram_rows_dist (launches)')
    wrap(_engine._PendingD, 'cpu', 'pending.cpu (wait + copy)')
    wrap(_engine, 'certified_selection', 'certified_selection')
    wrap(_engine.DeviceEngine, '_key_table', 'key_table (C++ walk)')
    wrap(ops.RowSet, 'from_virtual', 'RowSet.from_virtual')
    wrap(ops._PinnedRing, 'upload', 'pinned ring upload')
    wrap(ops, 'absent', 'absent')
    wrap(_engine.DeviceEngine, '_staged_rows', 'staged_rows')
    reps = 50
    walls, gpus = [], []
    # the selection too (krum_scores + the certificate), as aggregate()
    # runs it after the distance matrix
    def dm_and_select():
        D, st = agg.distance_matrix(fb)
        agg._certified_order(st, D, 10, 1, True)

    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        dm_and_select()
        e1.record()
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
        gpus.append(e0.elapsed_time(e1))
    walls.sort()
    gpus.sort()
    print(json.dumps({
        'what': 'KrumAggregator.distance_matrix + the certified '
                'selection, 50 x ConvNet2-h2048 device dicts',
        'wall_ms_median': walls[reps // 2],
        'event_ms_median': gpus[reps // 2],
        'path': agg.last_pairdist_path,
        'phases_us': {k: round(ACC[k] / CNT[k] * 1e6, 1) for k in ACC}}))


if __name__ == '__main__':
    main()
