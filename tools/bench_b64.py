#!/usr/bin/env python3
"""End-to-end rate of staging gRPC uploads (base64(pickle(tensor)) str
values, federatedscope/core/message.py:8-9) into the device client stack.

  host   the reference's decode per key (base64.b64decode + pickle.loads,
         core/auxiliaries/utils.py:95-105 — run here on fixtures this script
         pickled itself), then the pinned double-buffered H2D copy
  device core/compression/b64wire: framing walk on the host, the base64
         characters copied to pinned memory and DMA'd, fsagg_b64_unpack_f32
         decodes into the row

Prints one JSON line per mode: ms per upload and the fp32 parameter bytes
delivered per second.

    python tools/bench_b64.py --params 25000000 --uploads 8
"""
import argparse
import base64
import json
import os
import pickle
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--params', type=int, default=25_000_000)
    ap.add_argument('--keys', type=int, default=1)
    ap.add_argument('--uploads', type=int, default=8)
    ap.add_argument('--distinct', type=int, default=2)
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    from collections import OrderedDict
    from federatedscope_amd.core.compression import b64wire
    from federatedscope_amd.layout import BucketLayout, ClientStack, HostStager

    per = args.params // args.keys
    texts = []
    for d in range(args.distinct):
        g = torch.Generator().manual_seed(d)
        texts.append(OrderedDict(
            ('layer%d.weight' % j, base64.b64encode(pickle.dumps(
                torch.randn(per, generator=g))).decode())
            for j in range(args.keys)))
    chars = sum(len(v) for v in texts[0].values())
    lay = BucketLayout(OrderedDict((k, torch.zeros(per))
                                   for k in texts[0]))
    dev = torch.device('cuda', 0)
    st = ClientStack(lay, args.uploads, dev)
    ups = [texts[i % args.distinct] for i in range(args.uploads)]

    def host_path():
        sg = HostStager(dev)
        for i, u in enumerate(ups):
            dec = OrderedDict((k, pickle.loads(base64.b64decode(v)))
                              for k, v in u.items())
            sg.put(lay, dec, st.slab[i])
        sg.finish()

    def device_path():
        sg = HostStager(dev)
        for i, u in enumerate(ups):
            sg.put(lay, u, st.slab[i])
        sg.finish()

    ref = None
    for mode, fn in (('device', device_path), ('host', host_path)):
        fn()                                   # warm (pinned buffers)
        torch.cuda.synchronize()
        if ref is None:
            ref = st.slab[:args.uploads].clone()
        else:
            assert torch.equal(ref, st.slab[:args.uploads]), mode
        best = None
        for _ in range(args.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            best = t if best is None else min(best, t)
        ms = best * 1e3 / args.uploads
        print(json.dumps({
            'mode': mode, 'params': args.params, 'keys': args.keys,
            'uploads': args.uploads, 'b64_chars_per_upload': chars,
            'ms_per_upload': round(ms, 3),
            'param_GBps': round(4.0 * args.params / (ms * 1e6), 3),
            'b64_GBps': round(chars / (ms * 1e6), 3),
            'device_puts': b64wire.STATS['device_puts']}), flush=True)


if __name__ == '__main__':
    main()
