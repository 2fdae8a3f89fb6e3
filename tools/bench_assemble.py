#!/usr/bin/env python3
"""Strong-scaled FedAvg with the full result assembled on every rank
(block-cyclic parameter pieces, the in-place RCCL all-gather
of round j overlapped with the compute of round j+1 —
core/sharding.PipelinedAssembly).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P tools/bench_assemble.py

One JSON line on rank 0: whole-job GB/s (4·n·P algorithmic bytes over the
max-over-ranks step time) for the assembled result, and, from the same run,
the output-left-sharded time (no collective) for comparison.  Total work is
fixed (C3: 100 clients × 25M params split over the ranks): strong scaling.
Synthetic data as bench.py (counter hash, generated on the device).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def log(*a):
    print('[assemble]', *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--clients', type=int, default=100)
    ap.add_argument('--params', type=int, default=25_000_000,
                    help='total parameters (split over the ranks)')
    ap.add_argument('--chunks', type=int, default=4)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    args = ap.parse_args()

    from bench import sample_sizes
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import fedavg_weights
    from federatedscope_amd.core.sharding import PipelinedAssembly

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        dist.init_process_group('nccl', rank=rank, world_size=world,
                                device_id=dev)

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[local])

    n, P = args.clients, args.params
    pa = PipelinedAssembly(P, chunks=args.chunks)
    w = torch.tensor(fedavg_weights(sample_sizes(n)), dtype=torch.float32,
                     device=dev)
    pieces = []
    for j, (lo, hi) in enumerate(pa.local_pieces()):
        slab = torch.empty((n, pa.pc), dtype=torch.float32, device=dev)
        if hi > lo:
            ops.fill_uniform(slab, hi - lo, seed=2026, index_offset=lo)
        pieces.append(ops.RowTable.from_slab(slab, numel=max(hi - lo, 1)))
    out = torch.empty(pa.padded, dtype=torch.float32, device=dev)
    log('rank %d/%d: %d clients x %d params, %d rounds of %d-element pieces' %
        (rank, world, n, P, args.chunks, pa.pc))

    def compute(j, lo, hi, view):
        ops.weighted_sum(pieces[j], w, view)

    def sharded_only():
        for j, (lo, hi) in enumerate(pa.local_pieces()):
            if hi > lo:
                slot = (j * world + rank) * pa.pc
                compute(j, lo, hi, out[slot:slot + hi - lo])

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / args.steps
        if world > 1:
            tt = torch.tensor([t], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt.item())
        return t

    t_asm = timed(lambda: pa.run(compute, out=out))
    t_sh = timed(sharded_only)
    if rank == 0:
        rec = {
            'metric': 'aggregated-GB/s, FedAvg result assembled on every rank',
            'value': round(4.0 * n * P / t_asm / 1e9, 2),
            'unit': 'GB/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(t_asm * 1e3, 4),
            'higher_is_better': True, 'scaling': 'strong',
            'dtype': 'f32', 'data': 'synthetic (counter hash on device)',
            'config': {'workload': 'C3 FedAvg %d clients x %d params total, '
                                   'block-cyclic pieces, %d rounds, '
                                   'in-place all-gather per round' %
                                   (n, P, args.chunks),
                       'parallelism': 'param-range x%d + all-gather' % world},
            'sharded_only_ms': round(t_sh * 1e3, 4),
            'sharded_only_GBps': round(4.0 * n * P / t_sh / 1e9, 2),
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
