#!/usr/bin/env python3
"""Host cost of the row-set key table (csrc/host/keytable.cpp) for n device
dicts of the ConvNet2-h2048 layout (12 keys) and the ResNet-50 layout (161
keys): best-of-20 wall time per call.  GPU only (the table needs device
tensors)."""
import json
import os
import sys
import time
from collections import OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))

import torch  # noqa: E402
from bench_robust import CONVNET2_H2048  # noqa: E402
from federatedscope_amd import _lib  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    host = _lib.host()
    with open(os.path.join(ROOT, 'tools', 'resnet50_layout.json')) as f:
        r50 = [(k, tuple(s)) for k, s in json.load(f)['keys']]
    for name, layout, n in (('convnet2', CONVNET2_H2048, 200),
                            ('resnet50', r50, 100)):
        dicts = [OrderedDict((k, torch.empty(s, device=dev))
                             for k, s in layout) for _ in range(n)]
        keys = [k for k, _ in layout]
        shapes = [s for _, s in layout]
        offs = [0] * len(keys)
        for form, args in (('pointers', ()), ('virtual', (offs, ))):
            ts = []
            for _ in range(20):
                t0 = time.perf_counter()
                host.key_table(dicts, keys, shapes, dev.index, *args)
                ts.append(time.perf_counter() - t0)
            t = min(ts)
            print(json.dumps({'layout': name, 'clients': n,
                              'keys': len(keys), 'form': form,
                              'us_per_call': round(t * 1e6, 1),
                              'ns_per_tensor': round(
                                  t * 1e9 / (n * len(keys)), 1)}),
                  flush=True)


if __name__ == '__main__':
    main()
