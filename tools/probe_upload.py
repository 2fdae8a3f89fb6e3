#!/usr/bin/env python3
"""Host cost of one pinned-ring upload (ops._PinnedRing.upload), statement
by statement: the same calls timed in isolation over many repetitions of a
4.8-KB table (Krum's row table at C4).  GPU only."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def t(fn, reps=2000):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    dt = (time.perf_counter() - t0) / reps * 1e6
    torch.cuda.synchronize()
    return round(dt, 2)


def main():
    from federatedscope_amd import ops
    dev = torch.device('cuda', 0)
    arr = np.arange(600, dtype=np.int64)
    ring = ops._RING
    ring.upload(arr, dev)
    side = ring._copy_stream(dev)
    cur = torch.cuda.current_stream(dev)
    pinned = ring.buf[:arr.nbytes]
    d0 = torch.empty(arr.nbytes, dtype=torch.uint8, device=dev)
    ev = torch.cuda.Event()

    def ctx():
        with torch.cuda.stream(side):
            pass

    hip = ctypes.CDLL('libamdhip64.so')
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_void_p]
    hip.hipMemcpyAsync.restype = ctypes.c_int
    dst, src, nb = d0.data_ptr(), pinned.data_ptr(), arr.nbytes
    sh = side.cuda_stream

    def raw():
        # hipMemcpyHostToDevice = 1; the copy a native ring would issue
        rc = hip.hipMemcpyAsync(dst, src, nb, 1, sh)
        assert rc == 0, rc

    res = {
        'hipMemcpyAsync via ctypes (side stream)': t(raw),
        'upload (whole)': t(lambda: ring.upload(arr, dev)),
        'ops._h2d_np': t(lambda: ops._h2d_np(arr, dev)),
        'np.ascontiguousarray + view': t(
            lambda: np.ascontiguousarray(arr).reshape(-1).view(np.uint8)),
        'pinned slot write (numpy)': t(
            lambda: ring.np.__setitem__(slice(0, arr.nbytes),
                                        arr.view(np.uint8))),
        'torch.cuda.current_stream': t(lambda: torch.cuda.current_stream(dev)),
        'with torch.cuda.stream(side)': t(ctx),
        'torch.empty (device)': t(
            lambda: torch.empty(arr.nbytes, dtype=torch.uint8, device=dev)),
        'copy_ pinned->device non_blocking': t(
            lambda: d0.copy_(pinned, non_blocking=True)),
        'event.record': t(lambda: ev.record(side)),
        'tensor.record_stream': t(lambda: d0.record_stream(cur)),
        'stream.wait_event': t(lambda: cur.wait_event(ev)),
        'event.synchronize (done)': t(lambda: ev.synchronize()),
        'view + reshape': t(lambda: d0.view(torch.int64).reshape(600)),
    }
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
