#!/usr/bin/env python3
"""Host-side phases of the drop-in ClientsAvgAggregator.aggregate() on
device-resident ConvNet2-h2048 dicts (200 clients), or with --layout
resnet50 the configs[2] layout B dicts (100 clients, 161 keys, views of one
slab row per client, as bench.py's plugin_surface_layout_b): each phase
wrapped with perf_counter (no device synchronisation inside), mean
microseconds per call, plus the call's return time and its synchronised
wall time.  GPU only."""
import argparse
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
    static = isinstance(obj.__dict__.get(name), staticmethod)

    @functools.wraps(f)
    def g(*a, **kw):
        t0 = time.perf_counter()
        try:
            return f(*a, **kw)
        finally:
            ACC[label] += time.perf_counter() - t0
            CNT[label] += 1
    setattr(obj, name, staticmethod(g) if static else g)


def main():
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.core.aggregators import _engine
    ap = argparse.ArgumentParser()
    ap.add_argument('--layout', default='convnet2',
                    choices=['convnet2', 'resnet50'])
    ap.add_argument('--pipelined', action='store_true',
                    help='back-to-back calls without synchronising: a '
                         'phase that waits for the GPU shows the wait')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(7)
    cfg = SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=1000, sample_client_rate=1.0),
        aggregator=SimpleNamespace(byzantine_node_num=0, BFT_args=None))
    agg = ClientsAvgAggregator(device=dev, config=cfg)
    if args.layout == 'convnet2':
        fb = [(1 + i, OrderedDict((k, torch.randn(s, device=dev,
                                                  generator=g))
                                  for k, s in CONVNET2_H2048))
              for i in range(200)]
    else:
        from federatedscope_amd.layout import BucketLayout
        with open(os.path.join(ROOT, 'tools', 'resnet50_layout.json')) as f:
            keys = [(k, tuple(s)) for k, s in json.load(f)['keys']]
        lay = BucketLayout(OrderedDict((k, torch.empty(s, device='meta'))
                                       for k, s in keys))
        slab = torch.randn((100, ops.round_up(lay.numel, 64)), device=dev,
                           generator=g)
        fb = [(1 + i, OrderedDict(
            (k, slab[i, lay.offsets[k]:lay.offsets[k] + lay.numels[k]].view(
                lay.shapes[k])) for k in lay.keys)) for i in range(100)]
    info = {'client_feedback': fb, 'recover_fun': None}
    for _ in range(3):
        agg.aggregate(info)
    torch.cuda.synchronize()
    wrap(_engine.DeviceEngine, '_key_table', 'key_table')
    wrap(_engine.DeviceEngine, '_staged', 'staged (total)')
    wrap(_engine.DeviceEngine, '_run_pieces', 'run_pieces (kernel launch)')
    wrap(_engine.DeviceEngine, '_emit', 'emit')
    wrap(ops.RowSet, 'from_pointers', 'RowSet.from_pointers')
    wrap(ops, 'absent', 'absent')
    wrap(ops, 'weighted_sum_rows', 'weighted_sum_rows')
    wrap(_engine, 'fedavg_weights', 'fedavg_weights')
    wrap(ops._PinnedRing, 'upload', 'pinned ring upload')
    wrap(ops.RowSet, 'from_virtual', 'RowSet.from_virtual')
    wrap(ops, '_fp32_dev', '_fp32_dev')
    wrap(_engine.DeviceEngine, '_staged_rows', 'staged_rows')
    reps = 20
    ret = 0.0
    wall = 0.0
    for _ in range(reps):
        if not args.pipelined:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        agg.aggregate(info)
        t1 = time.perf_counter()
        if not args.pipelined:
            torch.cuda.synchronize()
        t2 = time.perf_counter()
        ret += t1 - t0
        wall += t2 - t0
    rec = {k: round(ACC[k] / reps * 1e6, 1) for k in ACC}
    rec['aggregate() return'] = round(ret / reps * 1e6, 1)
    rec['aggregate() synchronised wall'] = round(wall / reps * 1e6, 1)
    print(json.dumps(rec, indent=1))


if __name__ == '__main__':
    main()
