#!/usr/bin/env python3
"""Aggregation-engine benchmark (BASELINE.json metric).

A "step" is one FedAvg reduction (fsagg_weighted_sum_f32) of configs[2] of
BASELINE.json — 100 clients x 25,000,000 fp32 parameters, synthetic updates
already resident in HBM — whose FULL result ends up on every GPU.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py
--gpus N ..., or a bare ``bench.py --gpus N``, which starts its own N rank
processes) is STRONG scaling of that fixed model: rank r owns parameter
range r of every client and runs the full client loop over it
(bit-identical to one GPU: no arithmetic crosses GPUs).  By default (RCCL
group) the reducing kernel stores each output tile into every GPU's copy
over xGMI, then a flag barrier (core/sharding.py PeerAssembly); the
fallback cuts the range into ``chunks`` rounds of N block-cyclic pieces
whose all-gathers overlap the next round (PipelinedAssembly).
value = 4·n·P bytes / max-over-ranks step time.
Secondary fields: the same sharded compute with the output left sharded
(no collective), and the weak-scaling rate (every rank its own 100 x 25M).

Prints ONE JSON line on rank 0 (driver contract: DESIGN.md §6).
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
SEED = 2026


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


def host_cores():
    """CPU threads this process is granted.  The GPU box runs us on a share
    of a large machine (os.cpu_count() and the affinity mask count all of
    its CPUs) and states the share in OMP_NUM_THREADS."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get('OMP_NUM_THREADS', '')
    return min(n, int(omp)) if omp.isdigit() and int(omp) > 0 else n


def cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown CPU'


def cpu_baseline_leg(rows_slab, weights, P, n_sample, dev):
    """Time oracle/torch_cpu.py (the reference's per-key ``tmp = x*w;
    acc += tmp`` loop in torch CPU ops, clients_avg_aggregator.py:60-100)
    on the first ``n_sample`` clients at full width (25M params, the
    reference's shape class), at 1 thread (fed_runner.py:297-299) and at
    all of this process's cores; best of 3 after a warm-up.  The GPU kernel
    reduces the same clients with the same weights and must match bit for
    bit."""
    import torch
    from federatedscope_amd import ops
    from oracle.torch_cpu import para_weighted_avg_torch
    host = rows_slab[:n_sample, :P].cpu()
    models = [(0, {'w': host[i]}) for i in range(n_sample)]
    w = weights[:n_sample]
    ref_out = torch.empty(P, dtype=torch.float32, device=dev)
    ops.weighted_sum(ops.RowTable.from_slab(rows_slab, rows=range(n_sample),
                                            numel=P), w, ref_out)
    gpu = ref_out.cpu()
    prev = torch.get_num_threads()
    res = {}
    exact = True
    for threads in (1, host_cores()):
        torch.set_num_threads(threads)
        para_weighted_avg_torch(models[:2], w)      # warm-up
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            got = para_weighted_avg_torch(models, w)['w']
            ts.append(time.perf_counter() - t0)
        exact = exact and torch.equal(got, gpu)
        res[threads] = min(ts)
        log('cpu baseline %d thread(s): %.3f s -> %.3f GB/s' %
            (threads, res[threads], 4.0 * n_sample * P / res[threads] / 1e9))
    torch.set_num_threads(prev)
    return res, exact


def plugin_surface_leg(args, dev, slab, rows, sizes, w_dev, P, rounds=5,
                       calls=10):
    """The plugin surface at the headline config: the reference's
    ClientsAvgAggregator.aggregate(agg_info) (clients_avg_aggregator.py:
    19-35) on 100 device-resident 25M-parameter state_dicts (views of the
    bench's client rows, read in place), timed back to back against the
    bare kernel on the same rows — interleaved rounds, median per call —
    with the results compared bit for bit."""
    import statistics
    from types import SimpleNamespace

    import torch
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    n = len(sizes)
    clients = [(sizes[i], {'w': slab[i, :P]}) for i in range(n)]
    cfg = SimpleNamespace(federate=SimpleNamespace(ignore_weight=False,
                                                   use_ss=False))
    agg = ClientsAvgAggregator(device=dev, config=cfg)
    info = {'client_feedback': clients, 'recover_fun': None}
    flat = torch.empty(ops.round_up(P, 64), dtype=torch.float32, device=dev)

    def run_agg():
        return agg.aggregate(info)

    def run_flat():
        ops.weighted_sum(rows, w_dev, flat)

    for _ in range(3):
        res = run_agg()
        run_flat()
    torch.cuda.synchronize()
    exact = torch.equal(res['w'], flat[:P])
    t_agg, t_flat = [], []
    for _ in range(rounds):
        for fn, acc in ((run_agg, t_agg), (run_flat, t_flat)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(calls):
                fn()
            torch.cuda.synchronize()
            acc.append((time.perf_counter() - t0) / calls * 1e3)
    a, f = statistics.median(t_agg), statistics.median(t_flat)
    log('plugin surface: aggregate() %.4f ms/call, bare kernel %.4f ms '
        '(ratio %.4f), bit-exact %s' % (a, f, a / f, exact))
    return {
        'what': 'ClientsAvgAggregator.aggregate(agg_info) on %d device '
                'dicts x %d fp32 params, read in place; back-to-back calls, '
                'median of %d interleaved rounds of %d' % (n, P, rounds,
                                                           calls),
        'ms_per_call': round(a, 4),
        'GBps': round(4.0 * n * P / a / 1e6, 1),
        'bare_kernel_ms': round(f, 4),
        'ratio_vs_bare_kernel': round(a / f, 4),
        'bit_exact_vs_kernel': exact,
    }


def _interleaved(fns, rounds, calls):
    """Median ms per call of each function, timed back to back in
    interleaved rounds of ``calls`` calls."""
    import statistics

    import torch
    ts = [[] for _ in fns]
    for _ in range(rounds):
        for fn, acc in zip(fns, ts):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(calls):
                fn()
            torch.cuda.synchronize()
            acc.append((time.perf_counter() - t0) / calls * 1e3)
    return [statistics.median(t) for t in ts]


def plugin_fresh_leg(dev, slab, rows, sizes, w_dev, P, rounds=5, calls=10):
    """The plugin surface as a server round meets it: every call gets NEW
    client dicts (new tensor objects over the client rows) and the upload
    cache is off, so each call walks the tensors, builds and uploads its
    row table and weights like a round with freshly received uploads
    (parallel_runner.py:290-293 hands aggregate() a deepcopy per upload);
    against the bare kernel, interleaved, bit-exact."""
    from types import SimpleNamespace

    import torch
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    n = len(sizes)
    cfg = SimpleNamespace(federate=SimpleNamespace(ignore_weight=False,
                                                   use_ss=False))
    agg = ClientsAvgAggregator(device=dev, config=cfg)
    flat = torch.empty(ops.round_up(P, 64), dtype=torch.float32, device=dev)
    res = [None]
    # distinct dict lists of distinct tensor objects, built before the
    # timing (building 100 views costs ~0.3 ms of host time that is no part
    # of aggregate()), cycled through
    sets = [{'client_feedback': [(sizes[i], {'w': slab[i, :P]})
                                 for i in range(n)], 'recover_fun': None}
            for _ in range(8)]
    nxt = [0]

    def run_agg():
        info = sets[nxt[0] % len(sets)]
        nxt[0] += 1
        res[0] = agg.aggregate(info)

    def run_flat():
        ops.weighted_sum(rows, w_dev, flat)

    ring = ops._RING
    prev = ring.cache_on
    ring.cache_on = False
    uploads = ring.uploads
    try:
        for _ in range(3):
            run_agg()
            run_flat()
        torch.cuda.synchronize()
        exact = torch.equal(res[0]['w'], flat[:P])
        hits = ring.hits
        a, f = _interleaved((run_agg, run_flat), rounds, calls)
        # one isolated call (synchronised before and after), median of 9
        lat = []
        for _ in range(9):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run_agg()
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - t0) * 1e3)
        lat.sort()
        hits = ring.hits - hits
    finally:
        ring.cache_on = prev
    log('plugin surface, fresh dicts + upload cache off: aggregate() %.4f '
        'ms/call, bare kernel %.4f ms (ratio %.4f), isolated call %.4f ms, '
        'bit-exact %s, cache hits %d' % (a, f, a / f, lat[4], exact, hits))
    return {
        'what': 'ClientsAvgAggregator.aggregate(agg_info) on %d NEW device '
                'dicts x %d fp32 params per call (row table and weights '
                'walked and uploaded every call: upload cache off); '
                'back-to-back calls, median of %d interleaved rounds of %d; '
                'isolated call = synchronised before and after, median of 9'
                % (n, P, rounds, calls),
        'ms_per_call': round(a, 4),
        'GBps': round(4.0 * n * P / a / 1e6, 1),
        'bare_kernel_ms': round(f, 4),
        'ratio_vs_bare_kernel': round(a / f, 4),
        'isolated_call_ms': round(lat[4], 4),
        'upload_cache_hits': hits,
        'table_uploads_per_call': round((ring.uploads - uploads) /
                                        max(nxt[0], 1), 2),
        'bit_exact_vs_kernel': exact,
    }


CONVNET2_H512 = [  # configs[1]: cv/model/cnn.py:14-50, trainable keys
    ('conv1.weight', (32, 1, 5, 5)), ('conv1.bias', (32, )),
    ('bn1.weight', (32, )), ('bn1.bias', (32, )),
    ('conv2.weight', (64, 32, 5, 5)), ('conv2.bias', (64, )),
    ('bn2.weight', (64, )), ('bn2.bias', (64, )),
    ('fc1.weight', (512, 3136)), ('fc1.bias', (512, )),
    ('fc2.weight', (62, 512)), ('fc2.bias', (62, ))]


def c2_leg(dev, rounds=5, calls=20):
    """configs[1] (BASELINE.json): FEMNIST ConvNet2 (hidden 512, 12
    trainable keys, 1,690,238 fp32 params) x 100 clients, FedAvg on one
    GPU.  The clients are 100 device-resident state_dicts whose keys are
    separate allocations (a trained model's parameters); the bare row-set
    kernel (fsagg_weighted_sum_rows_f32 over their key table) against
    ClientsAvgAggregator.aggregate() on the same dicts, back to back, and
    the isolated call; checked bit-exact against each other."""
    from collections import OrderedDict
    from types import SimpleNamespace

    import torch
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.core.aggregators._engine import fedavg_weights
    n = 100
    sizes = sample_sizes(n, seed=1)
    w = fedavg_weights(sizes)
    g = torch.Generator(device=dev).manual_seed(SEED + 2)
    clients = [(sizes[i], OrderedDict(
        (k, torch.rand(s, device=dev, generator=g) * 2 - 1)
        for k, s in CONVNET2_H512)) for i in range(n)]
    P = sum(t.numel() for t in clients[0][1].values())
    cfg = SimpleNamespace(federate=SimpleNamespace(ignore_weight=False,
                                                   use_ss=False))
    agg = ClientsAvgAggregator(device=dev, config=cfg)
    info = {'client_feedback': clients, 'recover_fun': None}
    st = agg._staged(clients)
    rs = st.rows().persist()      # kept across the calls below
    w_dev = torch.tensor(w, dtype=torch.float32, device=dev)
    out = torch.empty(rs.layout.numel, dtype=torch.float32, device=dev)
    res = [None]

    def run_kernel():
        ops.weighted_sum_rows(rs, w_dev, out)

    def run_agg():
        res[0] = agg.aggregate(info)

    for _ in range(3):
        run_kernel()
        run_agg()
    torch.cuda.synchronize()
    lay = rs.layout
    exact = all(torch.equal(res[0][k].reshape(-1),
                            out[lay.offsets[k]:lay.offsets[k] +
                                lay.numels[k]]) for k in lay.keys)
    # per-launch kernel time on the launch stream (HIP events)
    evs = []
    st_ = torch.cuda.current_stream(dev)
    for _ in range(50):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(st_)
        run_kernel()
        b.record(st_)
        evs.append((a, b))
    torch.cuda.synchronize()
    kern = sorted(a.elapsed_time(b) for a, b in evs)
    k_ms = sum(kern) / len(kern)
    t_k, t_a = _interleaved((run_kernel, run_agg), rounds, calls)
    lat = []
    for _ in range(9):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_agg()
        torch.cuda.synchronize()
        lat.append((time.perf_counter() - t0) * 1e3)
    lat.sort()
    algo = 4.0 * n * P + 4.0 * P + 4.0 * n
    log('C2 (ConvNet2 h512, %d x %d, %d keys): kernel %.4f ms/launch '
        '(%.0f GB/s, %.3f of HBM), back to back %.4f ms; aggregate() %.4f '
        'ms/call, isolated %.4f ms; bit-exact %s' %
        (n, P, len(lay.keys), k_ms, algo / k_ms / 1e6,
         algo / k_ms / 1e6 / HBM_PEAK_GBS, t_k, t_a, lat[4], exact))
    del clients, info, st, rs
    return {
        'what': 'configs[1]: FedAvg over %d device-resident FEMNIST ConvNet2 '
                '(h=512) state_dicts, %d keys as separate allocations, %d '
                'fp32 params; kernel = fsagg_weighted_sum_rows_f32 over their '
                'key table (HIP events per launch, mean of 50); back to back '
                '= median of %d interleaved rounds of %d calls'
                % (n, len(CONVNET2_H512), P, rounds, calls),
        'clients': n,
        'params': P,
        'kernel_ms': round(k_ms, 4),
        'kernel_GBps': round(algo / k_ms / 1e6, 1),
        'kernel_frac_of_hbm': round(algo / k_ms / 1e6 / HBM_PEAK_GBS, 4),
        'kernel_back_to_back_ms': round(t_k, 4),
        'aggregate_ms_per_call': round(t_a, 4),
        'aggregate_GBps': round(4.0 * n * P / t_a / 1e6, 1),
        'aggregate_isolated_ms': round(lat[4], 4),
        'bit_exact_vs_kernel': exact,
    }


def plugin_layout_b_leg(dev, sizes, w_dev, rounds=5, calls=10,
                        separate=False):
    """configs[2] layout B: the same call on the ResNet-50 layout (161 keys,
    tools/resnet50_layout.json) — 100 device-resident multi-key state_dicts
    whose keys are views of one slab row per client laid out as the bucket
    (read in place; a uniform row set: the flat kernel over each client's
    range), or with ``separate`` every key its own allocation (a per-module
    state_dict: the multi-key row-set kernel) — against the bare flat
    kernel over the same slab rows, interleaved, every key compared bit for
    bit."""
    import statistics
    from collections import OrderedDict
    from types import SimpleNamespace

    import torch
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.layout import BucketLayout
    with open(os.path.join(ROOT, 'tools', 'resnet50_layout.json')) as f:
        keys = [(k, tuple(s)) for k, s in json.load(f)['keys']]
    lay = BucketLayout(OrderedDict((k, torch.empty(s, device='meta'))
                                   for k, s in keys))
    n, P = len(sizes), lay.numel
    ld = ops.round_up(P, 64)
    slab = torch.empty((n, ld), dtype=torch.float32, device=dev)
    ops.fill_uniform(slab, ld, seed=SEED + 1)
    clients = [(sizes[i], OrderedDict(
        (k, slab[i, lay.offsets[k]:lay.offsets[k] + lay.numels[k]].view(
            lay.shapes[k])) for k in lay.keys)) for i in range(n)]
    if separate:
        clients = [(s, OrderedDict((k, v.clone()) for k, v in d.items()))
                   for s, d in clients]
    cfg = SimpleNamespace(federate=SimpleNamespace(ignore_weight=False,
                                                   use_ss=False))
    agg = ClientsAvgAggregator(device=dev, config=cfg)
    info = {'client_feedback': clients, 'recover_fun': None}
    rows = ops.RowTable.from_slab(slab, numel=ld)
    flat = torch.empty(ld, dtype=torch.float32, device=dev)

    def run_agg():
        return agg.aggregate(info)

    def run_flat():
        ops.weighted_sum(rows, w_dev, flat)

    for _ in range(3):
        res = run_agg()
        run_flat()
    torch.cuda.synchronize()
    exact = all(torch.equal(res[k].reshape(-1), flat[
        lay.offsets[k]:lay.offsets[k] + lay.numels[k]]) for k in lay.keys)
    t_agg, t_flat = [], []
    for _ in range(rounds):
        for fn, acc in ((run_agg, t_agg), (run_flat, t_flat)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(calls):
                fn()
            torch.cuda.synchronize()
            acc.append((time.perf_counter() - t0) / calls * 1e3)
    a, f = statistics.median(t_agg), statistics.median(t_flat)
    log('layout B (%d keys, %d params, %s): aggregate() %.4f ms/call, bare '
        'flat kernel %.4f ms (ratio %.4f), bit-exact %s' %
        (len(keys), P, 'separate tensors' if separate else 'slab views', a,
         f, a / f, exact))
    del slab, rows, clients, info
    torch.cuda.empty_cache()
    return {
        'what': 'ClientsAvgAggregator.aggregate(agg_info) on %d device '
                'dicts of the ResNet-50 layout (%d keys, %d fp32 params; %s, '
                'read in place) against the flat kernel over the same '
                'values; median of %d interleaved rounds of %d calls' % (
                    n, len(keys), P,
                    'every key a separate allocation (row-set kernel)'
                    if separate else 'views of one slab row per client laid '
                    'out as the bucket (uniform row set: flat kernel)',
                    rounds, calls),
        'keys': len(keys),
        'params': P,
        'ms_per_call': round(a, 4),
        'GBps': round(4.0 * n * P / a / 1e6, 1),
        'bare_flat_kernel_ms': round(f, 4),
        'ratio_vs_bare_kernel': round(a / f, 4),
        'bit_exact_vs_kernel': exact,
    }


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


class Dist:
    """The job's process group: RCCL ("nccl") over xGMI when N > 1.  The
    gloo backend is for the multi-process tests on a one-GPU box (ranks
    then share the visible GPUs round-robin; collectives go through host
    memory, see core/sharding.Comm)."""

    def __init__(self, gpus, backend='nccl'):
        import torch
        import torch.distributed as dist
        self.dist = dist
        self.backend = backend
        self.world = int(os.environ.get('WORLD_SIZE', '1'))
        self.rank = int(os.environ.get('RANK', '0'))
        self.local = int(os.environ.get('LOCAL_RANK', '0'))
        if self.world != gpus:
            # a line must never claim a GPU count other than the one run
            log('error: --gpus %d but WORLD_SIZE %d' % (gpus, self.world))
            sys.exit(2)
        if backend == 'gloo':
            self.local %= max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(self.local)
        self.dev = torch.device('cuda', self.local)
        if self.world > 1:
            if backend == 'nccl':
                dist.init_process_group('nccl', rank=self.rank,
                                        world_size=self.world,
                                        device_id=self.dev)
            else:
                dist.init_process_group(backend, rank=self.rank,
                                        world_size=self.world)

    def barrier(self):
        if self.world > 1:
            if self.backend == 'nccl':
                self.dist.barrier(device_ids=[self.local])
            else:
                self.dist.barrier()

    def max(self, x):
        import torch
        if self.world == 1:
            return x
        dev = self.dev if self.backend == 'nccl' else 'cpu'
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


class _PeerPlan:
    """core/sharding.PeerAssembly behind PipelinedAssembly's interface (one
    round; compute(j, lo, hi, outs) gets the list of output addresses)."""

    def __init__(self, P, dev):
        from federatedscope_amd.core.sharding import PeerAssembly
        self.pp = PeerAssembly(P, device=dev)
        self.chunks = 1
        self.pcs = [self.pp.pc]
        self.padded = self.pp.padded
        self.streams = 1
        self.numel = P

    def local_pieces(self):
        return [self.pp.piece()]

    def local_numel(self):
        return self.pp.pc

    def piece(self, j, r=None):
        return self.pp.piece(r)

    def run(self, compute, out=None):
        return self.pp.run(lambda lo, hi, outs: compute(0, lo, hi, outs))

    def check(self):
        self.pp.check()

    def close(self):
        self.pp.close()


def pmc_child(args):
    """The traffic leg's profiled program: the C3 reduction a few times
    (its launches are what rocprofv3 --pmc counts)."""
    import torch
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import fedavg_weights
    dev = torch.device('cuda', 0)
    n, P = args.clients, args.params
    slab = torch.empty((n, ops.round_up(P, 64)), dtype=torch.float32,
                       device=dev)
    ops.fill_uniform(slab, P, seed=SEED)
    rows = ops.RowTable.from_slab(slab, numel=P)
    w = torch.tensor(fedavg_weights(sample_sizes(n)), dtype=torch.float32,
                     device=dev)
    out = torch.empty(ops.round_up(P, 64), dtype=torch.float32, device=dev)
    for _ in range(4):
        ops.weighted_sum(rows, w, out)
    torch.cuda.synchronize()


def live_traffic(args, kernel='wsum_f32_vec_kernel'):
    """roofline.traffic measured in THIS run: two rocprofv3 --pmc passes,
    FETCH_SIZE and WRITE_SIZE in separate runs (one TCC counter group
    each), over a child ``bench.py --pmc-child`` started before this
    process touches the GPU.  HBM bytes per launch with the gfx950
    correction of /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE
    counts half the bytes of 16-B-per-lane streaming reads (x2), WRITE_SIZE
    is exact; both in KiB.  Returns (bytes, note)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which('rocprofv3')
    if prof is None:
        return None, 'rocprofv3 not on PATH'
    tmp = tempfile.mkdtemp(prefix='fsagg_pmc_', dir='/tmp')
    env = dict(os.environ, TMPDIR='/tmp')
    kib = {}
    try:
        for ctr in ('FETCH_SIZE', 'WRITE_SIZE'):
            d = os.path.join(tmp, ctr)
            cmd = ['timeout', '-k', '10', '-s', 'KILL', '150', prof,
                   '--pmc', ctr, '--output-format', 'csv', '-d', d, '-o',
                   'run', '--', sys.executable, os.path.abspath(__file__),
                   '--pmc-child', '--clients', str(args.clients),
                   '--params', str(args.params)]
            r = subprocess.run(cmd, cwd='/tmp', env=env,
                               stdout=subprocess.DEVNULL,
                               stderr=subprocess.PIPE, timeout=200)
            if r.returncode != 0:
                return None, '%s pass exited %d: %s' % (
                    ctr, r.returncode, r.stderr.decode(
                        'utf-8', 'replace')[-300:])
            vals = []
            for path in glob.glob(os.path.join(d, '**',
                                               '*counter_collection.csv'),
                                  recursive=True):
                with open(path) as f:
                    for row in csv.DictReader(f):
                        if kernel in row.get('Kernel_Name', '') and \
                                row.get('Counter_Name') == ctr:
                            vals.append(float(row['Counter_Value']))
            if not vals:
                return None, 'no %s rows for %s' % (ctr, kernel)
            kib[ctr] = sum(vals) / len(vals)
    except (OSError, subprocess.SubprocessError) as e:
        return None, '%s: %s' % (type(e).__name__, e)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    read_b = kib['FETCH_SIZE'] * 1024 * 2
    write_b = kib['WRITE_SIZE'] * 1024
    return read_b + write_b, (
        'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of %s in '
        'this run: read %.4g B (FETCH_SIZE x2, gfx950 half count of 16-B '
        'reads) + write %.4g B per launch' % (kernel, read_b, write_b))


def free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(args, argv):
    """``--gpus N`` (N > 1) started without a launcher: start the N rank
    processes ourselves — one per GPU, RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set as torch.distributed.run sets them — the way the
    reference's parallel runner starts its own ranks
    (core/parallel/parallel_runner.py:89-96).  Runs before this process
    touches the GPU (torch.cuda.device_count() does not initialise HIP on
    this image) and never execs: the children are started, rank 0's JSON
    line reaches our stdout through the inherited descriptor, and we exit
    with the first failing rank's status.  With RCCL a rank per GPU is
    required: fewer visible GPUs than N is an error, never a smaller-N
    line."""
    import signal
    import subprocess
    import torch
    n = args.gpus
    visible = torch.cuda.device_count()
    if args.backend == 'nccl' and visible < n:
        log('error: --gpus %d needs %d visible GPUs, found %d' %
            (n, n, visible))
        return 3
    port = free_port()
    log('starting %d rank processes (%s, MASTER 127.0.0.1:%d)' %
        (n, args.backend, port))
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r),
                   WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen(
            [sys.executable, os.path.abspath(__file__)] + argv, env=env))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    old = signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    log('rank %d exited %d; stopping the others' %
                        (procs.index(p), code))
                    stop()
            time.sleep(0.05)
    finally:
        stop()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        signal.signal(signal.SIGTERM, old)
    return rc


def default_split(world):
    """Rounds' relative sizes of the strong-scaling pipeline (None: equal
    rounds).  DESIGN §7."""
    return None


def timed_steps(D, fn, steps, warmup):
    """W untimed steps, then K steps between barrier + synchronize pairs;
    returns the max-over-ranks seconds per step."""
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    return D.max((time.perf_counter() - t0) / steps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--clients', type=int, default=100)
    ap.add_argument('--params', type=int, default=25_000_000,
                    help='total model parameters (configs[2]: 25M), split '
                         'over the GPUs')
    ap.add_argument('--chunks', type=int, default=0,
                    help='pipeline rounds of the assembly (0: 1 on one GPU, '
                         '8 on two, 4 otherwise)')
    ap.add_argument('--streams', type=int, default=0,
                    help='side streams the pipeline pieces round-robin over '
                         '(0: by piece size, core/sharding.py SMALL_PIECE; '
                         '1: all on the current stream)')
    ap.add_argument('--split', default='auto',
                    help="rounds' relative sizes, e.g. 4/2/1/0.5 ('auto': "
                         'by world size, DESIGN §7; "uniform": equal)')
    ap.add_argument('--assembly', default='auto',
                    choices=['auto', 'p2p', 'rccl'],
                    help='how the result reaches every GPU (N > 1): p2p = '
                         'the reducing kernel stores into every GPU\'s copy '
                         'over xGMI + a flag barrier (core/sharding.py '
                         'PeerAssembly); rccl = pipelined in-place '
                         'all-gathers (PipelinedAssembly); auto = p2p on RCCL '
                         'process groups')
    ap.add_argument('--cpu-clients', type=int, default=20,
                    help='clients (full width) timed on the CPU baseline')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-plugin', action='store_true',
                    help='skip the ClientsAvgAggregator.aggregate() leg')
    ap.add_argument('--no-c2', action='store_true',
                    help='skip the configs[1] (FEMNIST ConvNet2) leg')
    ap.add_argument('--no-weak', action='store_true',
                    help='skip the secondary weak-scaling phase (N > 1)')
    ap.add_argument('--e2e', action='store_true',
                    help='also time host dicts -> aggregate() -> host dicts')
    ap.add_argument('--layout', default='flat', choices=['flat', 'resnet50'])
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'],
                    help='process-group backend (gloo: multi-process tests '
                         'on one GPU)')
    ap.add_argument('--no-pmc', action='store_true',
                    help='skip the live PMC traffic passes (roofline.traffic '
                         'null)')
    ap.add_argument('--pmc-child', action='store_true',
                    help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error('--gpus must be >= 1')
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(spawn_ranks(args, sys.argv[1:]))
    import torch
    if args.pmc_child:
        return pmc_child(args)
    # before this process touches the GPU: the profiled children must not
    # be started from a GPU-initialised process
    traffic, traffic_note = None, 'not measured (N > 1: per-rank pieces)'
    single = args.gpus == 1 and int(os.environ.get('WORLD_SIZE', '1')) == 1
    if single and args.no_pmc:
        traffic_note = 'skipped (--no-pmc)'
    elif single:
        log('roofline.traffic: two rocprofv3 --pmc passes (FETCH_SIZE, '
            'WRITE_SIZE) of the C3 kernel ...')
        traffic, traffic_note = live_traffic(args)
        log('traffic: %s (%s)' % (traffic, traffic_note))
    from federatedscope_amd import ops
    from federatedscope_amd.core.aggregators._engine import fedavg_weights
    from federatedscope_amd.core.sharding import PipelinedAssembly

    D = Dist(args.gpus, args.backend)
    world, rank, dev = D.world, D.rank, D.dev
    n, P = args.clients, args.params
    # rounds: the last round's gather is exposed.  Two GPUs share one
    # xGMI link pair, so their gather is slowest: 8 rounds (pieces of 1.56M
    # parameters still reduce at the one-launch rate); from 4 GPUs up the
    # pieces would shrink below that, 4 rounds
    chunks = args.chunks or (1 if world == 1 else 8 if world == 2 else 4)
    split = default_split(world) if args.split == 'auto' else (
        None if args.split == 'uniform' else
        [float(x) for x in args.split.split('/')])
    if split is not None and args.chunks:
        split = split[:args.chunks]
    assembly = args.assembly
    if assembly == 'auto':
        assembly = 'p2p' if world > 1 and args.backend == 'nccl' else 'rccl'
    pa = None
    if assembly == 'p2p' and world > 1:
        try:
            pa = _PeerPlan(P, dev)
        except Exception as e:          # no IPC / peer access: collective
            log('peer assembly unavailable (%s: %s); using the pipelined '
                'all-gather' % (type(e).__name__, e))
            assembly = 'rccl'
    if pa is None:
        pa = PipelinedAssembly(P, chunks=chunks, streams=args.streams or None,
                               split=split)
    chunks = pa.chunks
    sizes = sample_sizes(n)
    weights = fedavg_weights(sizes)
    w_dev = torch.tensor(weights, dtype=torch.float32, device=dev)
    log('rank %d/%d on %s: %d clients x %d params, %d round(s) of %s-param '
        'pieces on %d stream(s) (%.2f GB per rank)' %
        (rank, world, torch.cuda.get_device_name(dev), n, P, chunks, pa.pcs,
         pa.streams, 4.0 * n * pa.local_numel() / 1e9))

    # this rank's pieces of every client: global coordinates [lo, hi) of
    # the same counter-hash model at every N
    pieces = []
    for j, (lo, hi) in enumerate(pa.local_pieces()):
        slab = torch.empty((n, pa.pcs[j]), dtype=torch.float32, device=dev)
        if hi > lo:
            ops.fill_uniform(slab, hi - lo, seed=SEED, index_offset=lo)
        pieces.append((slab, ops.RowTable.from_slab(slab,
                                                    numel=max(hi - lo, 1))))
    out = torch.empty(pa.padded, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()

    # per-launch HIP events on the launch stream (the roofline's kernel time)
    events = []
    record = [False]

    def compute(j, lo, hi, view):
        if record[0]:
            # on the stream the piece is launched on (a side stream when the
            # pipeline uses them)
            st = torch.cuda.current_stream(dev)
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record(st)
            reduce_piece(j, view)
            b.record(st)
            events.append((a, b, hi - lo))
        else:
            reduce_piece(j, view)

    def reduce_piece(j, view):
        if isinstance(view, list):      # peer assembly: every GPU's copy
            ops.weighted_sum_bcast(pieces[j][1], w_dev, view)
        else:
            ops.weighted_sum(pieces[j][1], w_dev, view)

    result = [out]

    def step():
        result[0] = pa.run(compute, out=out)

    def sharded_only():
        for j, (lo, hi) in enumerate(pa.local_pieces()):
            if hi > lo:
                compute(j, lo, hi, out[lo:hi])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    record[0] = True
    t_step = timed_steps(D, step, args.steps, 0)
    record[0] = False
    launches = [(a.elapsed_time(b), m) for a, b, m in events]
    kern_ms = sum(t for t, _ in launches) / args.steps      # per rank
    mean_launch_ms = sum(t for t, _ in launches) / len(launches)
    mean_launch_p = sum(m for _, m in launches) / len(launches)
    kern_ms = D.max(kern_ms)
    # every rank's launch covers the same share (equal pieces): the slowest
    # rank's mean launch sets the job's kernel rate
    mean_launch_ms = D.max(mean_launch_ms)
    t_sharded = timed_steps(D, sharded_only, args.steps, args.warmup) \
        if world > 1 else t_step

    out = result[0]
    pa.check()
    # assembly check: columns of every rank's pieces (other ranks' too),
    # regenerated here and reduced by the same kernel, must equal what the
    # all-gather delivered, bit for bit
    ok = True
    probe = min(65536, max(pa.pcs))
    for j in range(chunks):
        for r in range(world):
            lo, hi = pa.piece(j, r)
            for a in sorted({lo, max(lo, hi - probe)}):
                b = min(a + probe, hi)
                if b <= a:
                    continue
                tmp = torch.empty((n, ops.round_up(b - a, 64)),
                                  dtype=torch.float32, device=dev)
                ops.fill_uniform(tmp, b - a, seed=SEED, index_offset=a)
                chk = torch.empty(ops.round_up(b - a, 4),
                                  dtype=torch.float32, device=dev)
                ops.weighted_sum(ops.RowTable.from_slab(tmp, numel=b - a),
                                 w_dev, chk)
                ok = ok and torch.equal(chk[:b - a], out[a:b])
    ok = D.max(0.0 if ok else 1.0) == 0.0

    algo_launch = 4.0 * n * mean_launch_p + 4.0 * mean_launch_p + 4.0 * n
    # N > 1: all ranks' launches together against N x the HBM peak (the
    # per-rank fraction is the same number)
    achieved = world * algo_launch / (mean_launch_ms / 1e3) / 1e9
    peak = world * HBM_PEAK_GBS
    value = 4.0 * n * P / t_step / 1e9
    log('step %.3f ms (kernels %.3f ms/rank, sharded-output step %.3f ms), '
        'launch %.3f ms -> %.0f GB/s, assembled result bit-exact: %s' %
        (t_step * 1e3, kern_ms, t_sharded * 1e3, mean_launch_ms, achieved,
         ok))

    plugin = plugin_b = plugin_bs = plugin_fresh = c2 = None
    if world == 1 and not args.no_plugin:
        plugin = plugin_surface_leg(args, dev, pieces[0][0], pieces[0][1],
                                    sizes, w_dev, P)
        plugin_fresh = plugin_fresh_leg(dev, pieces[0][0], pieces[0][1],
                                        sizes, w_dev, P)
        plugin_b = plugin_layout_b_leg(dev, sizes, w_dev)
        plugin_bs = plugin_layout_b_leg(dev, sizes, w_dev, separate=True)
    if world == 1 and not args.no_c2:
        c2 = c2_leg(dev)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        k = min(args.cpu_clients, n)
        log('cpu baseline: torch CPU op-for-op FedAvg, %d clients x %d '
            'params' % (k, P))
        res, exact = cpu_baseline_leg(pieces[0][0], weights, P, k, dev)
        cores = host_cores()
        cpu = {
            'value': round(4.0 * k * P / res[1] / 1e9, 3),
            'unit': 'GB/s',
            'cores': 1,
            'kind': 'port',
            'all_cores': {'cores': cores,
                          'value': round(4.0 * k * P / res[cores] / 1e9, 3)},
            'sample': ('oracle/torch_cpu.py: the reference loop of '
                       'clients_avg_aggregator.py:60-100 in torch %s CPU '
                       'ops (tmp = x*w; acc += tmp per client), on the first '
                       '%d of the same %d synthetic clients at full width '
                       '(%d params); torch.set_num_threads(1) as '
                       'fed_runner.py:299, and %d threads; best of 3; GPU '
                       'kernel on the same clients bit-exact: %s; host %s' %
                       (torch.__version__, k, n, P, cores, exact,
                        cpu_model())),
        }

    weak = None
    if world > 1 and not args.no_weak:
        del pieces
        torch.cuda.empty_cache()
        ld = ops.round_up(P, 64)
        slab = torch.empty((n, ld), dtype=torch.float32, device=dev)
        ops.fill_uniform(slab, P, seed=SEED, index_offset=rank * P)
        rows = ops.RowTable.from_slab(slab, numel=P)
        wout = torch.empty(ld, dtype=torch.float32, device=dev)
        t_weak = timed_steps(D, lambda: ops.weighted_sum(rows, w_dev, wout),
                             args.steps, args.warmup)
        weak = {'value': round(world * 4.0 * n * P / t_weak / 1e9, 2),
                'ms_per_step': round(t_weak * 1e3, 4),
                'what': 'every rank its own %d x %d (no collective)' %
                        (n, P)}
        del slab, rows

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
            'scaling': 'strong',
            'vs_baseline': None,
            'dtype': 'f32',
            'data': 'synthetic: counter-hash uniform[-1,1) generated on '
                    'device; sample sizes 1+hash(i) mod 1000',
            'config': {
                'workload': 'configs[2]: FedAvg weighted sum, %d clients x '
                            '%d fp32 params in total, param-range sharded '
                            'over %d GPU(s), full result assembled on every '
                            'GPU' % (n, P, world),
                'clients': n,
                'params': P,
                'parallelism': (
                    'param-range x%d, peer assembly: the reducing kernel '
                    'stores every output tile into all %d GPUs\' copies over '
                    'xGMI, then a flag barrier' % (world, world)
                    if assembly == 'p2p' else
                    'param-range x%d, %d pipelined all-gather rounds %s on '
                    '%d stream(s)' % (world, chunks, pa.pcs, pa.streams))
                if world > 1
                else 'single GPU',
            },
            'roofline': {
                'bound': 'hbm',
                'achieved': round(achieved, 1),
                'peak': peak,
                'unit': 'GB/s',
                'frac': round(achieved / peak, 4),
                'per_rank_launch_ms': round(mean_launch_ms, 4),
                'traffic': traffic,
                'traffic_over_algorithmic': round(traffic / algo_launch, 5)
                if traffic and world == 1 else None,
                'traffic_source': traffic_note,
            },
            'cpu_baseline': cpu,
            'per_rank_kernel_ms': round(kern_ms, 4),
            'exposed_assembly_ms': round(max(t_step * 1e3 - kern_ms, 0.0), 4),
            'sharded_output': {
                'ms_per_step': round(t_sharded * 1e3, 4),
                'value': round(4.0 * n * P / t_sharded / 1e9, 2)},
            'weak_scaling': weak,
            'plugin_surface': plugin,
            'plugin_surface_fresh': plugin_fresh,
            'configs_1_c2': c2,
            'plugin_surface_layout_b': plugin_b,
            'plugin_surface_layout_b_separate': plugin_bs,
            'assembled_bit_exact': ok,
        }
        print(json.dumps(rec), flush=True)
    if args.e2e and world == 1:
        del pieces
        torch.cuda.empty_cache()
        e2e_leg(args, dev, weights, sizes)
    if hasattr(pa, 'close'):
        pa.close()
    D.close()


if __name__ == '__main__':
    main()
