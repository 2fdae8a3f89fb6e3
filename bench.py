#!/usr/bin/env python3
"""Aggregation-engine benchmark (BASELINE.json metric).

A "step" is one FedAvg reduction (fsagg_weighted_sum_f32) over one batch of
synthetic client updates that are already resident in HBM: configs[2] of
BASELINE.json, 100 clients × 25,000,000 fp32 parameters per GPU.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py
--gpus N ...): FedAvg is per-coordinate, so every rank owns its own parameter
range (rank r generates indices [r·P, (r+1)·P) of the global model) and runs
the full client loop over it — no data-path collective, bit-exact, weak
scaling; value = Σ_ranks 4·n·P bytes ÷ max-over-ranks step time.

Prints ONE JSON line on rank 0 (see the driver contract in DESIGN.md).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = ('aggregated-GB/s device-resident (clients×params fp32), '
          '1/2/4/8 MI355X; % HBM roofline')
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md


def log(*a):
    print('[bench]', *a, file=sys.stderr, flush=True)


def mix64(z):
    m = (1 << 64) - 1
    z &= m
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & m
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & m
    z ^= z >> 31
    return z


def sample_sizes(n, seed=0):
    """sample sizes 1 + hash(seed, i) mod 1000."""
    return [1 + mix64(seed * 0x9E3779B97F4A7C15 + i + 1) % 1000
            for i in range(n)]


def cpu_baseline_leg(slab, n, P_sample, weights, out_dev):
    """Time the CPU oracle (a numpy port of _para_weighted_avg, one thread)
    on the first P_sample columns of the same synthetic clients; check the
    GPU result bit-exact on that sample."""
    import numpy as np
    import oracle
    host = slab[:, :P_sample].cpu().numpy()
    models = [(0, {'w': host[i]}) for i in range(n)]
    # ref weights are the reference's doubles; sizes do not matter here
    want = None
    times = []
    for rep in range(4):
        t0 = time.perf_counter()
        got = oracle.para_weighted_avg(models, weights=weights)
        times.append(time.perf_counter() - t0)
        want = got['w']
    t = min(times[1:]) if len(times) > 1 else times[0]
    gpu = out_dev[:P_sample].cpu().numpy()
    exact = bool(gpu.tobytes() == want.astype(np.float32).tobytes())
    return t, exact


def e2e_leg(args, dev, weights, sizes):
    """Host state_dicts in, host state_dict out, through the drop-in
    ClientsAvgAggregator (pinned double-buffered staging, H2D, kernel, D2H).
    Reported on its own JSON line; never the bench `value`."""
    from collections import OrderedDict
    from types import SimpleNamespace

    import torch
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    n = args.clients
    if args.layout == 'resnet50':
        with open(os.path.join(ROOT, 'tools', 'resnet50_layout.json')) as f:
            keys = [(k, tuple(s)) for k, s in json.load(f)['keys']]
    else:
        keys = [('w', (args.params, ))]
    P = sum(int(torch.Size(s).numel()) for _, s in keys)
    log('e2e: building %d host clients x %d params (%d keys)' %
        (n, P, len(keys)))
    g = torch.Generator().manual_seed(0)
    clients = [(sizes[i], OrderedDict((k, torch.rand(s, generator=g))
                                      for k, s in keys)) for i in range(n)]
    cfg = SimpleNamespace(federate=SimpleNamespace(ignore_weight=False,
                                                   use_ss=False))
    agg = ClientsAvgAggregator(device=dev, config=cfg)
    info = {'client_feedback': clients, 'recover_fun': None}
    agg.aggregate(info)
    ts = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = agg.aggregate(info)
        ts.append(time.perf_counter() - t0)
        log('e2e aggregate %.3f s' % ts[-1])
    # PCIe reference: one pinned 1 GB H2D
    host = torch.empty(2**28, dtype=torch.float32, pin_memory=True)
    d = torch.empty_like(host, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    h2d = host.numel() * 4 / (time.perf_counter() - t0) / 1e9
    t = min(ts)
    rec = {'e2e': {
        'what': 'ClientsAvgAggregator.aggregate, host dicts in/out',
        'layout': args.layout, 'clients': n, 'params': P,
        'keys': len(keys), 'seconds': round(t, 4),
        'GBps_algorithmic': round(4.0 * n * P / t / 1e9, 3),
        'pinned_h2d_GBps': round(h2d, 2),
        'host_threads': torch.get_num_threads(),
        'out_device': str(next(iter(out.values())).device)}}
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--clients', type=int, default=100)
    ap.add_argument('--params', type=int, default=25_000_000,
                    help='parameters per GPU (configs[2]: 25M)')
    ap.add_argument('--cpu-sample', type=int, default=5_000_000,
                    help='columns of the workload timed on the CPU baseline')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--e2e', action='store_true',
                    help='also time host dicts -> aggregate() -> host dicts')
    ap.add_argument('--layout', default='flat', choices=['flat', 'resnet50'])
    ap.add_argument('--traffic', default=os.path.join(
        ROOT, 'profiles', 'traffic_fedavg_c3.json'))
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import fedavg_weights

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        log('note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE' %
            (args.gpus, world))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        dist.init_process_group('nccl', rank=rank, world_size=world,
                                device_id=dev)

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[local])

    n, P = args.clients, args.params
    ld = ops.round_up(P, 64)
    log('rank %d/%d on %s: %d clients x %d params (%.2f GB)' %
        (rank, world, torch.cuda.get_device_name(dev), n, P, 4 * n * ld / 1e9))
    slab = torch.empty((n, ld), dtype=torch.float32, device=dev)
    ops.fill_uniform(slab, P, seed=2026, index_offset=rank * P)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    rows = ops.RowTable.from_slab(slab, numel=P)
    sizes = sample_sizes(n)
    weights = fedavg_weights(sizes)
    w_dev = torch.tensor(weights, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()

    def step():
        ops.weighted_sum(rows, w_dev, out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    t_step = wall / args.steps
    if world > 1:
        tt = torch.tensor([t_step], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_step = float(tt.item())
    algo_bytes = 4.0 * n * P + 4.0 * P + 4.0 * n  # read rows + write out + w
    value = world * 4.0 * n * P / t_step / 1e9
    achieved = algo_bytes / (kern_ms / 1e3) / 1e9
    log('step %.3f ms  kernel %.3f ms  achieved %.0f GB/s' %
        (t_step * 1e3, kern_ms, achieved))

    traffic = None
    if os.path.exists(args.traffic):
        try:
            with open(args.traffic) as f:
                tr = json.load(f)
            if tr.get('clients') == n and tr.get('params') == P:
                traffic = tr.get('hbm_bytes_per_launch')
        except (OSError, ValueError):
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        ps = min(args.cpu_sample, P)
        log('cpu baseline: numpy oracle, %d clients x %d params' % (n, ps))
        t_cpu, exact = cpu_baseline_leg(slab, n, ps, weights, out)
        import numpy
        np_version = numpy.__version__
        cpu_model = 'unknown CPU'
        try:
            with open('/proc/cpuinfo') as f:
                for line in f:
                    if line.startswith('model name'):
                        cpu_model = line.split(':', 1)[1].strip()
                        break
        except OSError:
            pass
        cpu = {
            'value': round(4.0 * n * ps / t_cpu / 1e9, 3),
            'unit': 'GB/s',
            'cores': 1,
            'kind': 'port',
            'sample': ('oracle.para_weighted_avg (numpy restatement of '
                       'clients_avg_aggregator.py:60-100, 1 thread like '
                       'fed_runner.py:299) on the first %d params of the '
                       'same %d synthetic clients; best of 3; GPU output '
                       'bit-exact on this sample: %s; host %s, numpy %s, '
                       'torch %s' % (ps, n, exact, cpu_model,
                                     np_version, torch.__version__)),
        }
        log('cpu baseline %.3f s -> %.3f GB/s, bit-exact=%s' %
            (t_cpu, cpu['value'], exact))

    if rank == 0:
        rec = {
            'metric': METRIC,
            'value': round(value, 2),
            'unit': 'GB/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(t_step * 1e3, 4),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'f32',
            'data': 'synthetic: counter-hash uniform[-1,1) generated on '
                    'device; sample sizes 1+hash(i) mod 1000',
            'config': {
                'workload': 'configs[2]: FedAvg weighted sum, %d clients x '
                            '%d fp32 params per GPU (param-range shard per '
                            'rank, no collective)' % (n, P),
                'clients': n,
                'params_per_gpu': P,
                'parallelism': 'param-range x%d' % world,
            },
            'roofline': {
                'bound': 'hbm',
                'achieved': round(achieved, 1),
                'peak': HBM_PEAK_GBS,
                'unit': 'GB/s',
                'frac': round(achieved / HBM_PEAK_GBS, 4),
                'traffic': traffic,
            },
            'cpu_baseline': cpu,
        }
        print(json.dumps(rec), flush=True)
    if args.e2e and world == 1:
        del slab, rows
        torch.cuda.empty_cache()
        e2e_leg(args, dev, weights, sizes)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
