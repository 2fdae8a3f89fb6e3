#!/usr/bin/env python3
"""Robust-rule kernels at BASELINE.json configs[3]/[4] sizes on one GPU.

  C4  Krum pairwise distances, 50 clients × 6,603,902 params (ConvNet2 h=2048
      layout, 12 keys), f = 10 — synthetic honest/Byzantine updates as
      SURVEY §8(d) specifies (margin-checked).
  C5  coordinate-wise median and trimmed mean (ratio 0.2 → k = 40), 200 clients
      × 6,603,902 params, N(0,1) with 10 % of clients ×100.

Prints one JSON line per kernel: device time (HIP events on the launch
stream), algorithmic GB/s = 4·n·P/t, fraction of the 8 TB/s HBM peak, and the
parity check done on the same inputs (test infrastructure: the CPU oracle on
sampled coordinates, an fp64 torch restatement for Krum's distances).
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from federatedscope_amd import ops  # noqa: E402
from federatedscope_amd.core.aggregators.krum_aggregator import \
    krum_scores  # noqa: E402
from federatedscope_amd.layout import BucketLayout  # noqa: E402

PEAK = 8000.0
CONVNET2_H2048 = [('conv1.weight', (32, 1, 5, 5)), ('conv1.bias', (32, )),
                  ('conv2.weight', (64, 32, 5, 5)), ('conv2.bias', (64, )),
                  ('bn1.weight', (32, )), ('bn1.bias', (32, )),
                  ('bn2.weight', (64, )), ('bn2.bias', (64, )),
                  ('fc1.weight', (2048, 3136)), ('fc1.bias', (2048, )),
                  ('fc2.weight', (62, 2048)), ('fc2.bias', (62, ))]


def log(*a):
    print('[robust]', *a, file=sys.stderr, flush=True)


def timed(fn, reps=15, warm_s=0.05):
    # untimed calls for warm_s seconds first: the GPU clocks ramp up from
    # idle over the first milliseconds of load (the first timed calls of a
    # cold process read up to 15 % slow)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        fn()
        torch.cuda.synchronize()
    ts = []
    for _ in range(reps + 1):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts[1:]), min(ts[1:])


def layout():
    from collections import OrderedDict
    return BucketLayout(OrderedDict((k, torch.empty(s)) for k, s in
                                    CONVNET2_H2048))


def krum_c4(dev, n=50, f=10):
    lay = layout()
    P = lay.numel
    g = torch.Generator(device=dev).manual_seed(1234)
    base = torch.randn(P, device=dev, generator=g)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(1234))
    byz = set(perm[:f].tolist())
    slab = torch.empty((n, P), device=dev)
    for r in range(n):
        z = torch.randn(P, device=dev, generator=g)
        if r in byz:
            slab[r] = 0.1 + 0.05 * z
        else:
            slab[r] = base + 0.01 * (1 + 0.05 * r) * z
    # zero the per-key padding so it adds nothing to the distances
    mask = torch.zeros(P, dtype=torch.bool, device=dev)
    for k in lay.keys:
        mask[lay.offsets[k]:lay.offsets[k] + lay.numels[k]] = True
    slab[:, ~mask] = 0
    rows = ops.RowTable.from_slab(slab)
    segs = lay.segments()
    D = ops.pairdist(rows, segs)
    med, mn = timed(lambda: ops.pairdist(rows, segs))
    Dh = D.cpu()
    # fp64 restatement (test infrastructure): per-key direct-difference norms
    ref = torch.zeros((n, n), dtype=torch.float64)
    for k in lay.keys:
        o, m = lay.offsets[k], lay.numels[k]
        X = slab[:, o:o + m].double()
        sq = torch.zeros((n, n), dtype=torch.float64, device=dev)
        for a in range(n):
            sq[a] = ((X - X[a]) ** 2).sum(1)
        ref += sq.sqrt().cpu()
    ref.fill_diagonal_(float('inf'))
    off = ~torch.eye(n, dtype=torch.bool)
    rel = ((Dh.double() - ref).abs() / ref)[off].max().item()
    s_gpu = krum_scores(Dh, f)
    s_ref = krum_scores(ref.float(), f)
    srt = torch.sort(s_ref.double())[0]
    margin = float((srt[1] - srt[0]) / srt[0])
    sel_gpu = torch.sort(s_gpu)[1][:5].tolist()
    sel_ref = torch.sort(s_ref)[1][:5].tolist()
    # the matrix-core path the aggregators take for n <= 64
    # (fsagg_pairgram_rows_f32: every key, D, flags and per-pair bounds)
    import numpy as np
    from federatedscope_amd.core.aggregators._engine import (
        _GRAM_TOL, certified_selection)
    rs = ops.RowSet(lay, np.array([[slab[i].data_ptr()] for i in range(n)],
                                  dtype=np.int64), dev, keepalive=(slab, ))

    def gram_D():
        buf, D_, ill_, B_, _, sq2_ = ops.pairgram_rows_dist(rs, _GRAM_TOL)
        return sq2_, D_, ill_, B_

    sq2, Dg, ill, Bg = gram_D()
    Dg, flags = Dg.cpu(), ill.cpu().numpy()
    Bg = Bg.cpu().numpy().astype(np.float64)
    Bg = np.maximum(Bg, Bg.T) + (2 * len(lay.keys) + 2) * 2.0 ** -24 * \
        np.where(np.isfinite(Dg.numpy()), Dg.numpy(), 0.0)
    sg = krum_scores(Dg, f)
    certified = certified_selection(Dg.numpy(), Bg, f, 5,
                                    torch.sort(sg)[1].numpy(), True)
    # per key: the Gram path's worst relative distance error, the predicted
    # bound at that pair and the conditioning (Σ|x'|² / d², centred on the
    # medoid) of the worst-conditioned pair
    sqg = sq2[0].cpu().numpy()
    errg = sq2[1].cpu().numpy()
    medoid = int(ref.clone().fill_diagonal_(0).sum(1).argmin())
    per_key = []
    for s_, k in enumerate(lay.keys):
        o, m = lay.offsets[k], lay.numels[k]
        X = slab[:, o:o + m].double()
        Y = X - X[medoid]
        mag = (Y * Y).sum(1).cpu().numpy()
        sq = torch.zeros((n, n), dtype=torch.float64, device=dev)
        for a in range(n):
            sq[a] = ((X - X[a]) ** 2).sum(1)
        sq = sq.cpu().numpy()
        offd = ~np.eye(n, dtype=bool)
        abserr = np.abs(sqg[s_] - sq)[offd]
        err = np.abs(np.sqrt(sqg[s_]) - np.sqrt(sq))[offd] / \
            np.sqrt(sq)[offd]
        F = ((mag[:, None] + mag[None, :]) / np.where(sq > 0, sq, np.inf))[
            offd]
        i = int(err.argmax())
        per_key.append({'key': k, 'len': m, 'max_rel_err': float(err[i]),
                        'F_at_max': float(F[i]), 'F_max': float(F.max()),
                        'err_over_F_max': float((err / F).max()),
                        # pairgram.hip: the worst-case bound err
                        'bound_holds': bool(np.all(
                            abserr <= errg[s_][offd])),
                        'max_abserr_over_bound': float(
                            (abserr / np.maximum(errg[s_][offd],
                                                 1e-300)).max()),
                        'max_abserr_over_G': float((abserr / np.maximum(
                            (mag[:, None] + mag[None, :])[offd],
                            1e-300)).max())})
    gmed, gmn = timed(gram_D)
    grel = ((Dg.double() - ref).abs() / ref)[off].max().item()
    sel_gram = torch.sort(krum_scores(Dg, f))[1][:5].tolist()
    # the drop-in: KrumAggregator's distance matrix on device dicts (views
    # of the slab rows, read in place), D back on the host
    from types import SimpleNamespace
    from federatedscope_amd.core.aggregators import KrumAggregator
    cfg = SimpleNamespace(
        federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                 client_num=1000, sample_client_rate=1.0),
        aggregator=SimpleNamespace(byzantine_node_num=f,
                                   BFT_args=SimpleNamespace(krum_agg_num=1)))
    agg = KrumAggregator(device=dev, config=cfg)
    models = [(1, {k: slab[i, lay.offsets[k]:lay.offsets[k] +
                            lay.numels[k]].view(lay.shapes[k])
                   for k in lay.keys}) for i in range(n)]
    De, _ = agg.distance_matrix(models)
    emed, emn = timed(lambda: agg.distance_matrix(models))
    erel = ((De.double() - ref).abs() / ref)[off].max().item()
    sel_eng = torch.sort(krum_scores(De, f))[1][:5].tolist()
    nbytes = 4.0 * n * P
    flops = 1.5 * n * (n - 1) * P
    return {
        'engine_ms_median': emed, 'engine_ms_min': emn,
        'engine_path': agg.last_pairdist_path,
        'engine_max_rel_err_vs_fp64': erel,
        'engine_selection_exact': sel_eng == sel_ref,
        'gram_ms_median': gmed, 'gram_ms_min': gmn,
        'gram_GBps': nbytes / gmed / 1e6,
        'gram_max_rel_err_vs_fp64': grel,
        'gram_flagged_pairs': int((flags > 0).sum()),
        'gram_max_rel_pair_bound': float((Bg / ref.numpy())[off.numpy()].max()),
        'gram_selection5_certified': bool(certified),
        'gram_per_key': per_key,
        'gram_selection_exact': sel_gram == sel_ref,
        'kernel': 'fsagg_pairdist_f32', 'config': 'C4 Krum n=%d P=%d f=%d' %
        (n, P, f), 'ms_median': med, 'ms_min': mn,
        'GBps': nbytes / med / 1e6, 'hbm_frac': nbytes / med / 1e6 / PEAK,
        'TFLOPs': flops / med / 1e9, 'fp32_vector_frac': flops / med / 1e9 /
        157.3, 'max_rel_err_vs_fp64': rel, 'score_margin': margin,
        'selection_exact': sel_gpu == sel_ref, 'selected': sel_gpu,
        'byzantine_selected': [i for i in sel_gpu if i in byz],
    }


def orderstat_c5(dev, n=200, ratio=0.2, P=None, tag='C5'):
    """``P`` given: a flat P-coordinate bucket instead of the C5 layout (the
    n > 255 sweep: the bit-by-bit select that re-reads columns from L2)."""
    P = layout().numel if P is None else int(P)
    g = torch.Generator(device=dev).manual_seed(2)
    slab = torch.randn((n, P), device=dev, generator=g)
    out_idx = torch.randperm(n, generator=torch.Generator().manual_seed(2))
    slab[out_idx[:n // 10]] *= 100.0
    rows = ops.RowTable.from_slab(slab)
    base = torch.randn(P, device=dev, generator=g)
    out = torch.empty(P, device=dev)
    k = int(n * ratio)
    res = []
    cols = torch.randperm(P, generator=torch.Generator().manual_seed(3))[:4096]
    cols = cols.sort()[0]
    host = slab[:, cols.to(dev)].cpu().numpy()
    hbase = base[cols.to(dev)].cpu().numpy()
    models = [(1, {'w': host[i]}) for i in range(n)]
    for name, fn in (('median', lambda: ops.coord_median(rows, out,
                                                          base=base)),
                     ('trimmed_mean', lambda: ops.trimmed_mean(rows, k, out,
                                                               base=base))):
        fn()
        torch.cuda.synchronize()
        got = out[cols.to(dev)].cpu().numpy()
        if name == 'median':
            want = oracle.median_aggregate(models, {'w': hbase})['w']
            ok = bool(got.tobytes() == want.tobytes())
            err = None
        else:
            want = oracle.add_init({'w': hbase},
                                   oracle.trimmed_mean_update(models, k))['w']
            eps = np.finfo(np.float32).eps
            err = float(np.max(np.abs(got - want)))
            grp = oracle.trimmed_group_bound(models, k)['w']
            ok = bool((np.abs(got.astype(np.float64) - want) <= grp + 4 * eps
                       * (np.abs(want) + np.abs(hbase) + 1e-30)).all())
        med, mn = timed(fn)
        nbytes = 4.0 * n * P + 8.0 * P
        res.append({
            'kernel': 'fsagg_%s_f32' % ('coord_median' if name == 'median'
                                        else name), 'config':
            '%s %s n=%d P=%d k=%d' % (tag, name, n, P, k if name != 'median'
                                      else 0), 'ms_median': med, 'ms_min': mn,
            'GBps': 4.0 * n * P / med / 1e6,
            'hbm_frac': nbytes / med / 1e6 / PEAK,
            'parity_sampled_4096_cols': ok, 'max_abs_err': err})
    return res


def dropin_rules(dev, fresh=False):
    """The drop-in aggregators' whole aggregate() call (Python, staging of the
    client dicts into the device stack, kernels, init + update) on
    device-resident ConvNet2-h2048 dicts (12 keys, 6.6M params): Krum
    (multi-Krum 5) and Bulyan at n = 50, f = 10; FedAvg, median, trimmed
    mean and norm bounding at n = 200.  Wall clock with the GPU synchronised on both
    sides; the result stays on the device.  ``fresh``: every call gets
    client tensors at addresses no earlier call used — each client key is a
    view at a new offset into a per-key pool, the way a server round's
    freshly received uploads are new tensors — so the clients' row tables
    are new every call (no upload-cache hit, no captured Gram chain to
    replay), while the server model and the layout's tables stay what they
    are in a real server (the same every round)."""
    from collections import OrderedDict
    from types import SimpleNamespace
    from federatedscope_amd.core.aggregators import (
        BulyanAggregator, ClientsAvgAggregator, KrumAggregator,
        MedianAggregator, NormboundingAggregator, TrimmedmeanAggregator)

    def cfg(f=0, agg_num=1, ratio=0.2, bound=5.0, client_num=1000):
        bft = SimpleNamespace(krum_agg_num=agg_num,
                              trimmedmean_excluded_ratio=ratio,
                              normbounding_norm_bound=bound)
        return SimpleNamespace(
            federate=SimpleNamespace(ignore_weight=False, use_ss=False,
                                     client_num=client_num,
                                     sample_client_rate=1.0),
            aggregator=SimpleNamespace(byzantine_node_num=f, BFT_args=bft),
            asyn=SimpleNamespace(staleness_discount_factor=1.0))

    class M(torch.nn.Module):
        def __init__(self, sd):
            super().__init__()
            self._sd = sd

        def state_dict(self, *a, **kw):
            # nn.Module.state_dict() hands out references, not copies
            return self._sd

    g = torch.Generator(device=dev).manual_seed(7)
    keys = [(k, s) for k, s in CONVNET2_H2048]
    init = OrderedDict((k, torch.randn(s, device=dev, generator=g))
                       for k, s in keys)
    P = sum(v.numel() for v in init.values())

    def clients(n):
        return [(int(1 + i), OrderedDict(
            (k, 1e-2 * torch.randn(s, device=dev, generator=g))
            for k, s in keys)) for i in range(n)]

    # fresh: per client and key a pool of numel + NOFF·64 values; call c of
    # rule r sees the key at offset 64·(30r + c) (16-B aligned, an address
    # no earlier call of any rule used)
    NWARM, NCALLS = 10, 20
    NOFF = 6 * (NWARM + NCALLS)

    def pools(n):
        return [[1e-2 * torch.randn(int(np.prod(s)) + 64 * NOFF,
                                    device=dev, generator=g)
                 for k, s in keys] for _ in range(n)]

    def fresh_sets(pool, r):
        first = r * (NWARM + NCALLS)
        return [[(int(1 + i), OrderedDict(
            (k, pool[i][j][64 * c:64 * c + int(np.prod(s))].view(s))
            for j, (k, s) in enumerate(keys))) for i in range(len(pool))]
            for c in range(first, first + NWARM + NCALLS)]

    out = []
    if fresh:
        c50, c200 = pools(50), pools(200)
    else:
        c50, c200 = clients(50), clients(200)
    rules = [
        ('fedavg', 200, ClientsAvgAggregator(model=M(init), device=dev,
                                             config=cfg())),
        ('krum_agg5', 50, KrumAggregator(model=M(init), device=dev,
                                         config=cfg(f=10, agg_num=5))),
        ('bulyan', 50, BulyanAggregator(model=M(init), device=dev,
                                        config=cfg(f=10, client_num=50))),
        ('median', 200, MedianAggregator(model=M(init), device=dev,
                                         config=cfg())),
        ('trimmed_mean', 200, TrimmedmeanAggregator(model=M(init),
                                                    device=dev,
                                                    config=cfg(ratio=0.2))),
        ('normbounding', 200, NormboundingAggregator(model=M(init),
                                                     device=dev,
                                                     config=cfg(bound=5.0))),
    ]
    for r, (name, n, agg) in enumerate(rules):
        fb = c50 if n == 50 else c200
        infos = [{'client_feedback': f, 'recover_fun': None}
                 for f in (fresh_sets(fb, r) if fresh else [fb])]
        it = [0]

        def call():
            agg.aggregate(infos[it[0] % len(infos)])
            it[0] += 1
        torch.cuda.synchronize()
        if fresh:
            for _ in range(NWARM):       # clocks up, one offset each
                call()
                torch.cuda.synchronize()
        else:
            w0 = time.perf_counter()
            while time.perf_counter() - w0 < 0.05:   # clocks up (timed)
                call()
                torch.cuda.synchronize()
        ts = []
        for _ in range(NCALLS):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            call()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        t = statistics.median(ts)
        same = None
        if fresh:
            # the same call repeated on one of those client sets (its tables
            # cached after the second sighting, the Gram chain replayed): the
            # kernels' time on exactly this placement, host caches warm
            for _ in range(3):
                agg.aggregate(infos[0])
            tw = []
            for _ in range(NCALLS):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                agg.aggregate(infos[0])
                torch.cuda.synchronize()
                tw.append(time.perf_counter() - t0)
            same = round(statistics.median(tw) * 1e3, 3)
        out.append({'rule': name, 'clients': n, 'params': P,
                    'ms_same_rows_repeated': same,
                    'pairdist_path': getattr(agg, 'last_pairdist_path',
                                             None),
                    'ms_aggregate': round(t * 1e3, 3),
                    'GBps_algorithmic': round(4.0 * n * P / t / 1e9, 1),
                    'fresh_uploads': bool(fresh),
                    'what': 'aggregate() on device-resident dicts read in '
                            'place (row sets), kernels + init+update' + (
                                '; client tensors at new addresses every '
                                'call (fresh uploads)' if fresh else '')})
        log('%s%s: %.2f ms' % (name, ' (fresh)' if fresh else '', t * 1e3))
    return out


def main():
    dev = torch.device('cuda', 0)
    which = sys.argv[1:] or ['krum', 'orderstat', 'dropin']
    if 'krum' in which:
        t0 = time.time()
        print(json.dumps(krum_c4(dev)), flush=True)
        log('krum done in %.1fs' % (time.time() - t0))
        torch.cuda.empty_cache()
    if 'krum_large' in which:
        # n > 64: the Gram path on projective-plane lines, C4's layout and byte
        # count per client
        for n in (100, 200, 256):
            t0 = time.time()
            print(json.dumps(krum_c4(dev, n=n, f=n // 5)), flush=True)
            log('krum n=%d done in %.1fs' % (n, time.time() - t0))
            torch.cuda.empty_cache()
    if 'orderstat' in which:
        for r in orderstat_c5(dev):
            print(json.dumps(r), flush=True)
        torch.cuda.empty_cache()
    if 'orderstat_large' in which:
        # n > 255 at the C5 byte count (4nP = 5.28 GB)
        for n in (300, 500):
            for r in orderstat_c5(dev, n=n, P=(200 * 6603904 // n) // 64 * 64,
                                  tag='n>255'):
                print(json.dumps(r), flush=True)
            torch.cuda.empty_cache()
    if 'dropin' in which:
        for r in dropin_rules(dev):
            print(json.dumps(r), flush=True)
    if 'dropin_fresh' in which:
        for r in dropin_rules(dev, fresh=True):
            print(json.dumps(r), flush=True)


if __name__ == '__main__':
    main()
