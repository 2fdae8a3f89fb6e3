#!/usr/bin/env python3
"""One GPU's share of the strong-scaled C3 FedAvg (bench.py --gpus N), on a
one-GPU box: the rank's pieces of every round reduced by the same kernel on
the same streams as PipelinedAssembly.run, with the RCCL all-gather replaced
by tools/emu_comm.EmuComm (its own stream, a spin for the link time of the
bytes the rank receives at an assumed per-GPU receive rate, plus a device
copy of those bytes).  Prints one JSON line per (world, split, rate).

    python tools/bench_share.py --world 8 --rates 0,350,450,550
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))

import torch  # noqa: E402


def parse_split(s):
    if s == 'uniform4':
        return None, 4
    if s.startswith('uniform'):
        return None, int(s[7:])
    if s.startswith('taper'):
        # taper<r>x<k>, e.g. taper0.5x4
        r, k = s[5:].split('x')
        from federatedscope_amd.core.sharding import tapered_split
        return tapered_split(int(k), float(r)), int(k)
    w = [float(x) for x in s.split('/')]
    return w, len(w)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--world', type=int, default=8)
    ap.add_argument('--rank', type=int, default=0)
    ap.add_argument('--clients', type=int, default=100)
    ap.add_argument('--params', type=int, default=25_000_000)
    ap.add_argument('--splits', default='uniform4,taper0.5x4,taper0.7x4,'
                    '4/3/2/1,1/3/3/1,uniform3,taper0.6x5')
    ap.add_argument('--rates', default='0,350,450,550',
                    help='emulated per-GPU receive GB/s (0: no gather)')
    ap.add_argument('--streams', type=int, default=0)
    ap.add_argument('--steps', type=int, default=30)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--copy', type=int, default=1)
    ap.add_argument('--p2p', action='store_true',
                    help='time the peer-assembly share instead: one bcast '
                         'launch over P/world writing `world` uncached local '
                         'buffers (stand-ins for the peers) + the barrier')
    ap.add_argument('--aggregate', action='store_true',
                    help='time rank 0\'s share of the plug-in path: '
                         'ClientsAvgAggregator.aggregate() sharded by '
                         'parameter range with the peer assembly (fused '
                         'broadcast into world uncached buffers, barrier, '
                         'copy-out of the assembled bucket, status check)')
    args = ap.parse_args()
    if args.aggregate:
        return aggregate_share(args)
    if args.p2p:
        return p2p_share(args)

    from bench import sample_sizes
    from emu_comm import EmuComm, sleep_cycles_per_us
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import fedavg_weights
    from federatedscope_amd.core.sharding import PipelinedAssembly

    dev = torch.device('cuda', 0)
    n, P, W = args.clients, args.params, args.world
    w = torch.tensor(fedavg_weights(sample_sizes(n)), dtype=torch.float32,
                     device=dev)
    cyc = sleep_cycles_per_us(dev)
    print('[share] _sleep: %.1f cycles/us' % cyc, file=sys.stderr)
    for spec in args.splits.split(','):
        split, chunks = parse_split(spec)
        for rate in [float(r) for r in args.rates.split(',')]:
            comm = EmuComm(W, args.rank, dev, rate_gbps=rate or None,
                           copy=bool(args.copy and rate), cyc_per_us=cyc)
            pa = PipelinedAssembly(P, chunks=chunks, comm=comm, split=split,
                                   streams=args.streams or None)
            pieces = []
            for j, (lo, hi) in enumerate(pa.local_pieces()):
                slab = torch.empty((n, pa.pcs[j]), dtype=torch.float32,
                                   device=dev)
                if hi > lo:
                    ops.fill_uniform(slab, hi - lo, seed=2026,
                                     index_offset=lo)
                pieces.append(ops.RowTable.from_slab(
                    slab, numel=max(hi - lo, 1)))
            out = torch.empty(pa.padded, dtype=torch.float32, device=dev)
            ev = []
            rec = [False]

            def compute(j, lo, hi, view):
                if rec[0]:
                    st = torch.cuda.current_stream(dev)
                    a = torch.cuda.Event(enable_timing=True)
                    b = torch.cuda.Event(enable_timing=True)
                    a.record(st)
                    ops.weighted_sum(pieces[j], w, view)
                    b.record(st)
                    ev.append((a, b))
                else:
                    ops.weighted_sum(pieces[j], w, view)

            for _ in range(args.warmup):
                pa.run(compute, out=out)
            torch.cuda.synchronize()
            rec[0] = True
            t0 = time.perf_counter()
            for _ in range(args.steps):
                pa.run(compute, out=out)
            torch.cuda.synchronize()
            t = (time.perf_counter() - t0) / args.steps
            kern = sum(a.elapsed_time(b) for a, b in ev) / args.steps
            print(json.dumps({
                'world': W, 'split': spec, 'pcs': pa.pcs,
                'streams': pa.streams, 'rate_GBps': rate,
                'step_ms': round(t * 1e3, 4),
                'kernel_ms_sum': round(kern, 4),
                'speedup_vs_1458us': round(1.458 / (t * 1e3), 2)}),
                flush=True)
            del pieces, out
            torch.cuda.empty_cache()


def p2p_share(args):
    """PeerAssembly's per-rank step on one GPU: the bcast kernel over this
    rank's P/world coordinates storing into `world` uncached buffers (own +
    stand-ins for the peers, all local here: on the node world-1 of them are
    xGMI stores), then the flag barrier (world 1)."""
    import ctypes
    from bench import sample_sizes
    from federatedscope_amd import _lib as L, ops
    from federatedscope_amd.core.aggregators._engine import fedavg_weights
    from federatedscope_amd.core.sharding import PeerAssembly
    dev = torch.device('cuda', 0)
    n, P, W = args.clients, args.params, args.world
    w = torch.tensor(fedavg_weights(sample_sizes(n)), dtype=torch.float32,
                     device=dev)
    pp = PeerAssembly(P // W, device=dev)      # world 1: own buffers only
    lib = L.load()
    fake = []
    for _ in range(W - 1):
        p = ctypes.c_void_p()
        L.check(lib.fsagg_peer_alloc(0, pp.padded * 4, ctypes.byref(p)))
        fake.append(int(p.value))
    slab = torch.empty((n, pp.pc), dtype=torch.float32, device=dev)
    ops.fill_uniform(slab, pp.numel, seed=2026, index_offset=0)
    rows = ops.RowTable.from_slab(slab, numel=pp.numel)
    for ndst in sorted({1, W}):
        ev = []

        def compute(lo, hi, outs):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            ops.weighted_sum_bcast(rows, w, (outs + fake)[:ndst])
            b.record()
            ev.append((a, b))

        for _ in range(args.warmup):
            pp.run(compute)
        torch.cuda.synchronize()
        ev.clear()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            pp.run(compute)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / args.steps
        pp.check()
        kern = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
        print(json.dumps({
            'mode': 'p2p-share', 'world': W, 'outputs': ndst,
            'share_params': pp.numel, 'step_ms': round(t * 1e3, 4),
            'kernel_ms': round(kern, 4),
            'kernel_TBps_in': round(4.0 * n * pp.numel / kern / 1e9, 3),
            'speedup_vs_1458us': round(1.458 / (t * 1e3), 2)}), flush=True)
    for p in fake:
        lib.fsagg_peer_free(0, p)
    pp.close()


def aggregate_share(args):
    """Rank ``--rank`` of ``world`` through Aggregator.aggregate() on one
    GPU: the engine's sharded path (``aggregator.shard_by_param_range``)
    with a PeerAssembly whose world - 1 peer copies are local uncached
    buffers and whose barrier waits for this rank alone — everything that
    rank does on the node (its row table over the 100 device dicts, the
    reduction of its P/world range stored into every copy, the barrier, the
    result, the status check), without the xGMI link time.

    Per mode one JSON line:
      latency   — synchronize, one aggregate(), synchronize (median);
      pipelined — 10 back-to-back calls between synchronizes (per call);
    for the default result (a fresh copy of the assembled bucket, status
    checked before returning) and ``shard_result_views`` (views of the
    rotating copies, status checked at the next call); with the upload
    cache on (the same client tensors every call, as a persistent client
    model gives) and off (every table uploaded, as new client tensors
    would need)."""
    import ctypes
    import statistics
    from types import SimpleNamespace
    from bench import sample_sizes
    from federatedscope_amd import _lib as L, ops
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.core.sharding import Comm, PeerAssembly
    dev = torch.device('cuda', 0)
    n, P, W, R = args.clients, args.params, args.world, args.rank
    lib = L.load()

    class EmuPeers(PeerAssembly):
        def __init__(self, numel, buffers):
            super().__init__(numel, comm=Comm(), device=dev,
                             buffers=buffers)   # world 1
            self.world = W
            self.rank = R
            self.pc = max(-(-numel // W // 64) * 64, 64)
            self.fake = []
            for _ in range(W - 1):
                q = ctypes.c_void_p()
                L.check(lib.fsagg_peer_alloc(0, self.padded * 4,
                                             ctypes.byref(q)))
                self.fake.append(int(q.value))
            own = self._ptr[0]
            self._ptr = [[q] * len(own) for q in self.fake[:R]] + [own] + \
                [[q] * len(own) for q in self.fake[R:]]

        def _barrier(self):
            saved, sr = self.world, self.rank
            self.world, self.rank = 1, 0
            saved_flags = self._flags
            self._flags = (ctypes.c_void_p * 1)(self._ptr[sr][-1])
            try:
                super()._barrier()
            finally:
                self.world, self.rank = saved, sr
                self._flags = saved_flags

        def free(self):
            for q in self.fake:
                lib.fsagg_peer_free(0, q)
            self.world = 1

    sizes = sample_sizes(n)
    slab = torch.empty((n, -(-P // 64) * 64), dtype=torch.float32,
                       device=dev)
    ops.fill_uniform(slab, P, seed=2026)
    clients = [(sizes[i], {'w': slab[i, :P]}) for i in range(n)]
    cfg = SimpleNamespace(federate=SimpleNamespace(ignore_weight=False,
                                                   use_ss=False))
    ref = torch.empty(-(-P // 64) * 64, dtype=torch.float32, device=dev)
    ops.weighted_sum(ops.RowTable.from_slab(slab, numel=P),
                     [s / sum(sizes) for s in sizes], ref)
    info = {'client_feedback': clients, 'recover_fun': None}

    def measure(agg):
        for _ in range(args.warmup):
            agg.aggregate(info)
        torch.cuda.synchronize()
        lat = []
        for _ in range(args.steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = agg.aggregate(info)
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - t0) * 1e3)
        pipe = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                out = agg.aggregate(info)
            torch.cuda.synchronize()
            pipe.append((time.perf_counter() - t0) * 1e3 / 10)
        return statistics.median(lat), statistics.median(pipe), out

    base = None
    for world, views in [(1, False)] + [(W, v) for v in (False, True)]:
        for cache in ((True, ) if world == 1 else (True, False)):
            ops._RING.cache_on = cache
            ops._RING.clear()
            agg = ClientsAvgAggregator(device=dev, config=cfg)
            emu = None
            if world > 1:
                emu = EmuPeers(P, 3 if views else 2)
                layout = agg._staged_rows(clients).layout
                agg.cfg = SimpleNamespace(
                    federate=cfg.federate, aggregator=SimpleNamespace(
                        shard_by_param_range=True, shard_chunks=1,
                        shard_assembly='p2p', shard_result_views=views))
                agg._shard = lambda: (emu.comm, 1)
                agg._plans[(layout.signature(), 1, 'p2p', views)] = emu
            lat, pipe, out = measure(agg)
            ok = None
            if world > 1:
                lo, hi = emu.piece()
                ok = bool(torch.equal(out['w'][lo:hi], ref[lo:hi]))
                emu.check()
                emu.free()
            else:
                base = lat
            print(json.dumps({
                'mode': 'aggregate-share', 'world': world, 'rank': R,
                'clients': n, 'params': P,
                'result': ('views' if views else 'copy') if world > 1
                else 'unsharded', 'upload_cache': cache,
                'ms_latency': round(lat, 4), 'ms_pipelined': round(pipe, 4),
                'piece_bit_exact': ok,
                'speedup_latency_vs_world1': round(base / lat, 2)}),
                flush=True)
    ops._RING.cache_on = True


if __name__ == '__main__':
    main()
