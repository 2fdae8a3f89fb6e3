#!/usr/bin/env python3
"""Host cost of rank 0's sharded ClientsAvgAggregator.aggregate() (peer
assembly emulated on one GPU as in tools/bench_share.py --aggregate): the
wall time of the call's host side alone (no synchronize inside the timed
loop, GPU work queued behind), and a cProfile of 200 calls by total time."""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))


def main():
    import argparse
    import torch
    ap = argparse.ArgumentParser()
    ap.add_argument('--views', type=int, default=1)
    ap.add_argument('--params', type=int, default=25_000_000)
    a = ap.parse_args()
    import ctypes
    from types import SimpleNamespace
    from bench import sample_sizes
    from federatedscope_amd import _lib as L, ops
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.core.sharding import Comm, PeerAssembly
    dev = torch.device('cuda', 0)
    lib = L.load()
    n, P, W = 100, a.params, 8
    pa = PeerAssembly(P, comm=Comm(), device=dev, buffers=3)
    pa.world = W
    pa.pc = max(-(-P // W // 64) * 64, 64)
    fake = []
    for _ in range(W - 1):
        q = ctypes.c_void_p()
        L.check(lib.fsagg_peer_alloc(0, pa.padded * 4, ctypes.byref(q)))
        fake.append(int(q.value))
    own = pa._ptr[0]
    pa._ptr = [own] + [[q] * len(own) for q in fake]
    flags1 = (ctypes.c_void_p * 1)(own[-1])
    real_barrier = PeerAssembly._barrier

    def barrier1(self):
        self.world, fl = 1, self._flags
        self._flags = flags1
        try:
            real_barrier(self)
        finally:
            self.world, self._flags = W, fl
    pa._barrier = barrier1.__get__(pa)
    sizes = sample_sizes(n)
    slab = torch.empty((n, -(-P // 64) * 64), dtype=torch.float32,
                       device=dev)
    ops.fill_uniform(slab, P, seed=2026)
    clients = [(sizes[i], {'w': slab[i, :P]}) for i in range(n)]
    cfg = SimpleNamespace(federate=SimpleNamespace(ignore_weight=False,
                                                   use_ss=False))
    agg = ClientsAvgAggregator(device=dev, config=cfg)
    layout = agg._staged_rows(clients).layout
    agg.cfg = SimpleNamespace(federate=cfg.federate, aggregator=SimpleNamespace(
        shard_by_param_range=True, shard_chunks=1, shard_assembly='p2p',
        shard_result_views=bool(a.views)))
    agg._shard = lambda: (pa.comm, 1)
    agg._plans[(layout.signature(), 1, 'p2p', bool(a.views))] = pa
    info = {'client_feedback': clients, 'recover_fun': None}
    for _ in range(20):
        agg.aggregate(info)
    torch.cuda.synchronize()
    ts = []
    for _ in range(50):
        t0 = time.perf_counter()
        agg.aggregate(info)
        ts.append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize()
    ts.sort()
    print('host us per aggregate(): median %.1f min %.1f (views=%d)' %
          (ts[len(ts) // 2], ts[0], a.views))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200):
        agg.aggregate(info)
        torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats('tottime').print_stats(25)
    print(s.getvalue())
    pa.check()
    for q in fake:
        lib.fsagg_peer_free(0, q)
    pa.world = 1


if __name__ == '__main__':
    main()
