#!/usr/bin/env python3
"""Host cost of one ClientsAvgAggregator.aggregate() call on the ResNet-50
layout (161 keys x 100 device clients, bench.py's layout-B legs): wall time
of the call without a sync (the host part; the kernel is async), the key-table
walk alone, the result unpack alone, and cProfile's top entries.  tools only.
"""
import cProfile
import json
import os
import pstats
import io
import statistics
import sys
import time
from collections import OrderedDict
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.layout import BucketLayout
    dev = torch.device('cuda', 0)
    with open(os.path.join(ROOT, 'tools', 'resnet50_layout.json')) as f:
        keys = [(k, tuple(s)) for k, s in json.load(f)['keys']]
    lay = BucketLayout(OrderedDict((k, torch.empty(s, device='meta'))
                                   for k, s in keys))
    n, P = 100, lay.numel
    ld = ops.round_up(P, 64)
    slab = torch.rand((n, ld), device=dev)
    for separate in (False, True):
        clients = [(1 + i, OrderedDict(
            (k, slab[i, lay.offsets[k]:lay.offsets[k] + lay.numels[k]].view(
                lay.shapes[k])) for k in lay.keys)) for i in range(n)]
        if separate:
            clients = [(s, OrderedDict((k, v.clone()) for k, v in d.items()))
                       for s, d in clients]
        cfg = SimpleNamespace(federate=SimpleNamespace(ignore_weight=False,
                                                       use_ss=False))
        agg = ClientsAvgAggregator(device=dev, config=cfg)
        info = {'client_feedback': clients, 'recover_fun': None}
        for _ in range(3):
            agg.aggregate(info)
        torch.cuda.synchronize()
        host, iso = [], []
        for _ in range(20):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            agg.aggregate(info)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            host.append((t1 - t0) * 1e3)
            iso.append((t2 - t0) * 1e3)
        dicts = [m for _, m in clients]
        kt = []
        for _ in range(20):
            t0 = time.perf_counter()
            agg._key_table(lay if not separate else agg._fast_layouts[
                (tuple(dicts[0].keys()), False)], dicts, virtual=True)
            kt.append((time.perf_counter() - t0) * 1e3)
        flat = torch.empty(P, device=dev)
        up = []
        for _ in range(20):
            t0 = time.perf_counter()
            agg._emit(lay, flat, list(dicts[0].keys()), dev)
            up.append((time.perf_counter() - t0) * 1e3)
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(10):
            agg.aggregate(info)
        pr.disable()
        torch.cuda.synchronize()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats('tottime').print_stats(14)
        print(json.dumps({
            'separate': separate,
            'host_ms_per_call': round(statistics.median(host), 4),
            'isolated_ms_per_call': round(statistics.median(iso), 4),
            'key_table_ms': round(statistics.median(kt), 4),
            'emit_ms': round(statistics.median(up), 4)}), flush=True)
        print(s.getvalue(), file=sys.stderr, flush=True)
        del clients, info, agg
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
