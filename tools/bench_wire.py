#!/usr/bin/env python3
"""End-to-end rates of the §8(f) rows on one GPU (one JSON line each).

  quant  100 clients × ResNet-50 layout (23.5M params, 161 keys) uploaded as
         int8 wire dicts (conv/fc weights quantised, the rest fp32) through
         AggregationServer(stage_on_arrival, dequantize): pinned pack → one
         H2D per upload (~1 B per quantised param) → fsagg_wire_unpack_f32 →
         FedAvg.  Compared with the same uploads as fp32 dicts (4 B/param).
  ss     secret-sharing FedAvg recovery (fsagg_ss_recover_f32) over 100
         parties' int64/float64 share sums of 6M coordinates, device-resident.
  dissim calc_l2_dissim + calc_blocal_dissim over 100 × 6M staged clients.

Synthetic data (int codes / shares drawn uniformly); timings are wall clock
around the whole call with the GPU synchronised on both sides.
"""
import json
import os
import sys
import time
from collections import OrderedDict
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def log(*a):
    print('[wire]', *a, file=sys.stderr, flush=True)


def cfg(use_ss=False):
    return SimpleNamespace(federate=SimpleNamespace(
        ignore_weight=False, use_ss=use_ss, client_num=1000,
        sample_client_rate=1.0))


class _Model(torch.nn.Module):
    def state_dict(self, *a, **kw):
        return OrderedDict()

    def load_state_dict(self, sd, strict=True):
        pass


def resnet_keys():
    with open(os.path.join(ROOT, 'tools', 'resnet50_layout.json')) as f:
        return [(k, tuple(s)) for k, s in json.load(f)['keys']]


def quant_leg(n=100, reps=2):
    from federatedscope_amd.core.aggregators import ClientsAvgAggregator
    from federatedscope_amd.core.compression.utils import dequantize_tensor
    from federatedscope_amd.core.workers.server import AggregationServer
    keys = resnet_keys()
    g = torch.Generator().manual_seed(5)
    wires, fp32s = [], []
    qparams = 0
    P = 0
    for i in range(n):
        w = OrderedDict()
        for k, s in keys:
            numel = int(torch.Size(s).numel())
            if i == 0:
                P += numel
            if ('fc' in k or 'conv' in k) and k.split('.')[-1] == 'weight':
                w[k.replace('weight', 'weight_quant')] = torch.randint(
                    -127, 128, s, dtype=torch.int8, generator=g)
                w[k.replace('weight', 'weight_scale')] = torch.tensor(
                    1e-3 * (1 + i % 7), dtype=torch.float32)
                if i == 0:
                    qparams += numel
            else:
                w[k] = torch.randn(s, generator=g)
        wires.append((int(1 + (i * 37) % 500), w))
    log('quant: %d clients, %d params, %d quantised' % (n, P, qparams))
    wire_bytes = sum(v.numel() * v.element_size() for v in wires[0][1].values())
    def run(stage_quant):
        srv = AggregationServer(_Model(), ClientsAvgAggregator(config=cfg()),
                                sample_client_num=n, stage_on_arrival=True,
                                dequantize=stage_quant)
        ts = []
        for r in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for sender, (s, w) in enumerate(wires if stage_quant else fp32s):
                srv.callback_funcs_model_para(r, sender, (s, w))
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return min(ts[1:])

    t_q = run(True)
    log('quant staged: %.3f s' % t_q)
    # fp32 uploads of the same model (dequantised on the host once, outside
    # the timed region)
    for s, w in wires:
        d = OrderedDict()
        for k, v in w.items():
            if 'weight_quant' in k:
                d[k.replace('weight_quant', 'weight')] = dequantize_tensor(
                    v, w[k.replace('weight_quant', 'weight_scale')])
            elif 'weight_scale' in k:
                continue
            else:
                d[k] = v
        fp32s.append((s, d))
    t_f = run(False)
    log('fp32 staged: %.3f s' % t_f)
    return {'leg': 'quant_e2e', 'clients': n, 'params': P,
            'quantised_params': qparams, 'wire_bytes_per_upload': wire_bytes,
            'seconds_int8_wire': round(t_q, 4),
            'seconds_fp32_wire': round(t_f, 4),
            'GBps_algorithmic_int8': round(4.0 * n * P / t_q / 1e9, 2),
            'GBps_algorithmic_fp32': round(4.0 * n * P / t_f / 1e9, 2),
            'wire_GBps_int8': round(n * wire_bytes / t_q / 1e9, 2),
            'speedup': round(t_f / t_q, 2),
            'what': 'AggregationServer.callback_funcs_model_para x n '
                    '(stage on arrival) + FedAvg; host dicts in, device '
                    'result out'}


def ss_leg(n=100, P=6_000_000):
    from federatedscope_amd import ops
    dev = torch.device('cuda')
    g = torch.Generator(device=dev).manual_seed(3)
    shares = []
    for i in range(n):
        if i % 3:
            shares.append(torch.randint(-2**62, 2**62, (P, ), device=dev,
                                        dtype=torch.int64, generator=g))
        else:
            shares.append(torch.randint(0, 2**61, (P, ), device=dev,
                                        dtype=torch.int64,
                                        generator=g).double())
    mod = float(2 * 2**60 + 1)
    ops.ss_recover(shares, mod, float(2**60), 1e8, 12345.0)
    ts = []
    for _ in range(5):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.ss_recover(shares, mod, float(2**60), 1e8, 12345.0)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 1e3)
    t = min(ts)
    nbytes = 8.0 * n * P + 4.0 * P
    return {'leg': 'ss_recover', 'parties': n, 'params': P,
            'ms': round(t * 1e3, 3), 'GBps': round(nbytes / t / 1e9, 1),
            'hbm_frac': round(nbytes / t / 1e9 / 8000.0, 4),
            'what': 'fsagg_ss_recover_f32 incl. row-table upload, '
                    'device-resident shares'}


def dissim_leg(n=100, P=6_000_000):
    from federatedscope_amd.core.monitors import (calc_blocal_dissim,
                                                  calc_l2_dissim)
    dev = torch.device('cuda')
    keys = [('conv.weight', (P // 2, )), ('fc.weight', (P - P // 2, ))]
    g = torch.Generator(device=dev).manual_seed(4)
    last = OrderedDict((k, torch.randn(s, device=dev, generator=g))
                       for k, s in keys)
    clients = [(int(1 + i), OrderedDict(
        (k, v + 1e-2 * torch.randn(v.shape, device=dev, generator=g))
        for k, v in last.items())) for i in range(n)]
    calc_l2_dissim(last, clients)
    out = {}
    for name, fn in (('l2', calc_l2_dissim), ('blocal', calc_blocal_dissim)):
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn(last, clients)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name + '_ms'] = round(min(ts) * 1e3, 2)
    # kernels alone (HIP events): the fused B-local pass against the two
    # passes it replaces, on the same key table
    from federatedscope_amd import ops
    kt = ops.KeyTable([list(m.values()) for _, m in clients], dev)
    base = list(last.values())
    w = [1.0 / n] * n
    gbuf = torch.empty(kt.numel, device=dev)

    def two_pass():
        ops.delta_sqnorm_keys(kt, base=base)
        ops.delta_wsum_keys(kt, w, base, gbuf)

    def fused():
        ops.delta_sqnorm_wsum_keys(kt, w, base, gbuf)
    for name, fn in (('blocal_two_pass_kernels', two_pass),
                     ('blocal_fused_kernels', fused),
                     ('blocal_two_pass_kernels', two_pass),
                     ('blocal_fused_kernels', fused)):
        fn()
        ts = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[name + '_ms'] = round(min(out.get(name + '_ms', 1e9),
                                      sorted(ts)[len(ts) // 2]), 3)
    return dict(leg='dissim', clients=n, params=P, **out,
                what='device-resident client dicts read in place (ops.KeyTable) + metric kernels')


def main():
    legs = sys.argv[1:] or ['quant', 'ss', 'dissim']
    for leg in legs:
        rec = {'quant': quant_leg, 'ss': ss_leg, 'dissim': dissim_leg}[leg]()
        print(json.dumps(rec), flush=True)
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
