#!/usr/bin/env python3
"""Interleaved A/B timing of weighted-sum variants (rows in flight U ×
float4 columns per lane V × nt loads × grid) on N × P (default 100 × 25M;
rows at a 256-B aligned leading dimension), plus the
read-only stream ceiling.  Prints one line per variant: median/min ms and
GB/s.  GPU only; run through tools/gpu_job.sh."""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from federatedscope_amd import _lib, ops  # noqa: E402

VARIANTS = {0: 'U8V2nt', 1: 'U2V8nt', 2: 'U4V8nt', 3: 'U1V8nt', 4: 'U2V16nt',
            5: 'U1V16nt', 6: 'U4V4nt', 7: 'U3V8nt', 8: 'U2V8', 9: 'U1V12nt',
            10: 'U1V20nt', 11: 'U1V24nt', 12: 'U1V1nt', 13: 'U4V1nt',
            14: 'U8V1nt', 15: 'U2V4nt', 16: 'U1V4nt', 17: 'U4V2nt'}

PART = {0: 'U1V8', 1: 'U1V12', 2: 'U1V16', 3: 'U1V24', 4: 'U2V8', 5: 'U2V12',
        6: 'U1V32', 7: 'U4V4'}


def main():
    n = int(os.environ.get('N', 100))
    P = int(os.environ.get('P', 25_000_000))
    rounds = int(os.environ.get('ROUNDS', 7))
    lib = _lib.load()
    lib.fsagg_tune_wsum.argtypes = [ctypes.c_int, ctypes.c_uint,
                                    ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_int, ctypes.c_int64,
                                    ctypes.c_void_p, ctypes.c_void_p]
    lib.fsagg_tune_wsum_part.argtypes = lib.fsagg_tune_wsum.argtypes
    lib.fsagg_tune_readbw.argtypes = [ctypes.c_int, ctypes.c_uint,
                                      ctypes.c_void_p, ctypes.c_int64,
                                      ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device('cuda', 0)
    # rows 256-B aligned as every staged or bench slab lays them out
    ld = ops.round_up(P, 64)
    slab = torch.empty((n, ld), dtype=torch.float32, device=dev)
    ops.fill_uniform(slab, ld, seed=1)
    rows = ops.RowTable.from_slab(slab, numel=P)
    w = torch.full((n, ), 1.0 / n, dtype=torch.float32, device=dev)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    ref = torch.empty_like(out)
    ops.weighted_sum(rows, w, ref)
    st = torch.cuda.current_stream().cuda_stream
    red = torch.empty(256 * 16 * 256 * 4, dtype=torch.float32, device=dev)
    grids = [int(g) for g in os.environ.get('GRIDS', '0,2048').split(',')]
    cases = []
    for v in [int(x) for x in os.environ.get('VARS', ','.join(
            str(k) for k in VARIANTS)).split(',')]:
        for g in grids:
            cases.append(('wsum', v, g))
    for v in ([int(x) for x in os.environ['PVARS'].split(',')]
              if os.environ.get('PVARS') is not None and os.environ['PVARS']
              else ([] if 'PVARS' in os.environ else PART)):
        for g in [int(x) for x in os.environ.get(
                'PGRIDS', '256,512,768,1024,2048').split(',')]:
            cases.append(('part', v, g))
    for nt in ((0, 1) if not os.environ.get('NOREAD') else ()):
        for g in (4096, 8192, 16384):
            cases.append(('read', nt, g))
    times = {c: [] for c in cases}
    for r in range(rounds):
        for c in cases:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            if c[0] == 'part':
                _lib.check(lib.fsagg_tune_wsum_part(c[1], c[2], rows.ptr(),
                                                    w.data_ptr(), n, P,
                                                    out.data_ptr(), st),
                           'tune_part')
            elif c[0] == 'wsum':
                _lib.check(lib.fsagg_tune_wsum(c[1], c[2], rows.ptr(),
                                               w.data_ptr(), n, P,
                                               out.data_ptr(), st), 'tune')
            else:
                _lib.check(lib.fsagg_tune_readbw(c[1], c[2], slab.data_ptr(),
                                                 n * ld, red.data_ptr(), st),
                           'readbw')
            e1.record()
            e1.synchronize()
            times[c].append(e0.elapsed_time(e1))
            if r == 0 and c[0] in ('wsum', 'part'):
                assert torch.equal(out, ref), c
        print('round', r, 'done', file=sys.stderr, flush=True)
    for c in cases:
        t = times[c][1:]
        med, mn = statistics.median(t), min(t)
        nbytes = 4.0 * n * P + (4.0 * P if c[0] != 'read' else 0)
        name = {'wsum': VARIANTS, 'part': PART}[c[0]][c[1]] \
            if c[0] != 'read' else ('read nt=%d' % c[1])
        print('%-5s %-10s grid=%-5d med %.3f ms min %.3f ms  %.0f GB/s (med)'
              % (c[0], name, c[2], med, mn, nbytes / med / 1e6))


if __name__ == '__main__':
    main()
