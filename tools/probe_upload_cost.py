#!/usr/bin/env python3
"""Host cost of one small table upload (ops._PinnedRing.upload with the
cache off) and of its parts, on the GPU box: µs per call, median of 5
rounds of 2000.  tools only."""
import statistics
import sys
import os
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def per_call(fn, n=2000, rounds=5):
    ts = []
    for _ in range(rounds):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        ts.append((time.perf_counter() - t0) / n * 1e6)
        torch.cuda.synchronize()
    return round(statistics.median(ts), 2)


def main():
    from federatedscope_amd import ops
    dev = torch.device('cuda', 0)
    ring = ops._RING
    ring.cache_on = False
    arr = np.arange(100, dtype=np.int64)
    side = torch.cuda.Stream(device=dev)
    cur = torch.cuda.current_stream(dev)
    ev = torch.cuda.Event()
    pinned = torch.empty(1 << 20, dtype=torch.uint8, pin_memory=True)
    res = {
        'upload_persistent_cache_off': per_call(lambda: ring.upload(arr, dev)),
        'upload_ephemeral_ring': per_call(
            lambda: ring.upload(arr, dev, ephemeral=True)),
    }

    def ctx():
        with torch.cuda.stream(side):
            pass
    res['stream_ctx'] = per_call(ctx)
    res['empty'] = per_call(lambda: torch.empty(800, dtype=torch.uint8,
                                                device=dev))
    d = torch.empty(800, dtype=torch.uint8, device=dev)
    res['slice_copy_'] = per_call(lambda: d.copy_(pinned[0:800],
                                                  non_blocking=True))
    res['event_record'] = per_call(lambda: ev.record(side))
    res['record_stream'] = per_call(lambda: d.record_stream(cur))
    res['wait_event'] = per_call(lambda: cur.wait_event(ev))
    res['np_copy_into_pinned'] = per_call(
        lambda: pinned.numpy().__setitem__(slice(0, 800), arr.view(np.uint8)))
    ring.cache_on = True
    import json
    print(json.dumps(res))


if __name__ == '__main__':
    main()
