#!/usr/bin/env python3
"""Host cost of staging 200 device dicts (ConvNet2-h2048, 12 keys) for a
robust drop-in: _stage_all, and its parts — the native key walk, the row
set's construction — median µs over 300 calls.  tools only."""
import os
import statistics
import sys
import time
from collections import OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import torch  # noqa: E402
from bench_robust import CONVNET2_H2048  # noqa: E402
from profile_rule import M, cfg  # noqa: E402


def t(fn, k=300):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(k):
        a = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - a) * 1e6)
    return statistics.median(ts)


def main():
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators import MedianAggregator
    from federatedscope_amd.core.aggregators._engine import _host_ext
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(7)
    init = OrderedDict((k, torch.randn(s, device=dev, generator=g))
                       for k, s in CONVNET2_H2048)
    models = [(1 + i, OrderedDict((k, torch.randn(s, device=dev, generator=g))
                                  for k, s in CONVNET2_H2048))
              for i in range(200)]
    agg = MedianAggregator(model=M(init), device=dev, config=cfg(f=10))
    st = agg._stage_all(models)
    lay = st.layout
    dicts = [m for _, m in models]
    h = _host_ext()
    kl = lay.__dict__['_key_list']
    print('stage_all        %7.1f us' % t(lambda: agg._stage_all(models)))
    print('_key_table       %7.1f us' % t(
        lambda: agg._key_table(lay, dicts, virtual=True)))
    print('host.key_table   %7.1f us' % t(
        lambda: h.key_table(dicts, kl[0], kl[1], dev.index, kl[2])))
    kt = agg._key_table(lay, dicts, virtual=True)
    print('RowSet           %7.1f us' % t(
        lambda: ops.RowSet.from_virtual(lay, kt[0], dev, keepalive=(dicts,),
                                        missing=0, uniform=kt[3],
                                        ephemeral=True)))
    print('dict list        %7.1f us' % t(lambda: [m for _, m in models]))
    print('_base            %7.1f us' % t(
        lambda: agg._base(lay, agg.model.state_dict(), as_float=True)))
    print('state_dict       %7.1f us' % t(lambda: agg.model.state_dict()))
    rs = st.rows()
    out = torch.empty(lay.numel, device=dev)

    def launch():
        r2 = ops.RowSet.from_virtual(lay, kt[0], dev, keepalive=(dicts,),
                                     missing=0, uniform=kt[3],
                                     ephemeral=True)
        ops.coord_median_rows(r2, out)
    print('rowset+launch    %7.1f us' % t(launch, 100))
    torch.cuda.synchronize()


if __name__ == '__main__':
    main()
