#!/usr/bin/env python3
"""A/B at C5 (200 × 6.6M fp32, flat rows): the two-wave kernel (default)
against the K-wave kernel opened below 256 clients
(fsagg_orderstat_set_group_range / _waves), K = 4 and 8, for the median
and the trimmed mean (k = 40): interleaved rounds, median of 15 event-timed
calls per round after a clock warm-up; results checked against the
default kernel (median bit-exact, trimmed mean within 4e-6 relative).
tools only.  usage: [GROUP_KS=5,6,8] ab_group_small.py [n]"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    from federatedscope_amd import _lib as L
    from federatedscope_amd import ops
    lib = L.load()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    P = (200 * 6603904 // n) // 64 * 64
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(3)
    X = torch.randn((n, P), device=dev, generator=g)
    X[torch.rand((n, P), device=dev, generator=g) < 0.02] *= 100.0
    rows = ops.RowTable.from_slab(X)
    out = torch.empty(P, device=dev)
    k = int(0.2 * n)

    def variant(name):
        if name == 'pair':
            lib.fsagg_orderstat_set_group_range(-1, 0)
            lib.fsagg_orderstat_set_group_waves(0)
        else:
            lib.fsagg_orderstat_set_group_range(65, 512)
            lib.fsagg_orderstat_set_group_waves(int(name[5:]))

    def run(mode):
        if mode == 'median':
            ops.coord_median(rows, out)
        else:
            ops.trimmed_mean(rows, k, out)

    def timed(mode):
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        ts = []
        for _ in range(15):
            e0.record()
            run(mode)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return statistics.median(ts)

    # GROUP_KS=5,6,8 picks the K-wave variants (default 4, 8); 'pair' is the
    # library default at this n (the two-wave kernel below 256 clients, the
    # streaming or K-wave kernel above)
    ks = os.environ.get('GROUP_KS', '4,8').split(',')
    names = ['pair'] + ['group%s' % x for x in ks]
    ref = {}
    for mode in ('median', 'trimmed'):
        variant('pair')
        run(mode)
        ref[mode] = out.clone()
        for nm in names:
            variant(nm)
            run(mode)
            if mode == 'median':
                ok = bool(torch.equal(out, ref[mode]))
            else:
                ok = bool(((out - ref[mode]).abs() <=
                           4e-6 * ref[mode].abs() + 1e-6).all())
            print(json.dumps({'n': n, 'mode': mode, 'variant': nm,
                              'matches_default': ok}), flush=True)
    res = {}
    for rnd in range(3):
        for mode in ('median', 'trimmed'):
            for nm in names if rnd % 2 == 0 else names[::-1]:
                variant(nm)
                torch.cuda.synchronize()
                for _ in range(20):
                    run(mode)
                res.setdefault((mode, nm), []).append(timed(mode))
    variant('pair')
    for (mode, nm), v in sorted(res.items()):
        print(json.dumps({'n': n, 'mode': mode, 'variant': nm,
                          'ms_rounds': [round(x, 4) for x in v],
                          'ms_median': round(statistics.median(v), 4)}),
              flush=True)


if __name__ == '__main__':
    main()
