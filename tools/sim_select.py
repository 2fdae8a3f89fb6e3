#!/usr/bin/env python3
"""Lane-level Python model of the octave-digit select kernel
(federatedscope_amd/csrc/orderstat_select.hip), for debugging its index
arithmetic on the CPU: one column at a time, the same digits, intervals,
refinement plans, compaction and list positions.  Not test infrastructure
for parity (tests compare the GPU with oracle/); a development aid.

usage: sim_select.py N_CLIENTS  (runs the all-kernels test columns)
"""
import sys

import numpy as np

M32 = 0xFFFFFFFF


def ukey(u):
    s = M32 if u & 0x80000000 else 0
    return u ^ (s | 0x80000000)


def key2f(k):
    u = (k & 0x7FFFFFFF) if k & 0x80000000 else (~k & M32)
    return float(np.array([u], np.uint32).view(np.float32)[0])


def octave_digit(u, base):
    m = (u >> 20) & 0x7FF
    t = min(max(m - base, 0), 127)
    s = M32 if u & 0x80000000 else 0
    return ((t ^ s) + 128) & M32


def octave_bin(d, base):
    pos = d >= 128
    t = d - 128 if pos else 127 - d
    mlo = 0 if t == 0 else base + t
    mhi = 2047 if t == 127 else base + t
    alo = max(mlo, 0) << 20
    ahi = (max(mhi, 0) << 20) | 0xFFFFF
    if pos:
        return alo | 0x80000000, min(ahi | 0x80000000, 0xFF800000)
    return max((~(ahi | 0x80000000)) & M32, 0x007FFFFF), \
        (~(alo | 0x80000000)) & M32


def scan(hist, r):
    """digit holding rank r, count below it, count in it"""
    cum = 0
    for d, c in enumerate(hist):
        if cum + c > r:
            return d, cum, c
        cum += c
    raise AssertionError('rank %d past %d keys' % (r, cum))


def select(col, n, kk, median):
    u = [int(x) for x in np.asarray(col, np.float32).view(np.uint32)]
    amax = max(x & 0x7FFFFFFF for x in u)
    base = (amax >> 20) - 127
    r1 = (n - 1) // 2 if median else kk
    r2 = n // 2 if median else n - kk - 1
    h = [0] * 256
    for x in u:
        h[octave_digit(x, base)] += 1
    d1, b1, c1 = scan(h, r1)
    d2, b2, c2 = scan(h, r2)
    s1 = list(octave_bin(d1, base)) + [b1, c1]
    s2 = list(octave_bin(d2, base)) + [b2, c2]
    shared = s1[:2] == s2[:2]
    for rnd in range(10):
        l1 = s1[0] != s1[1]
        l2 = not shared and s2[0] != s2[1]
        stored = (s1[3] if l1 else 0) + (s2[3] if l2 else 0)
        if stored <= 32:
            break
        pick2 = l2 and (not l1 or s2[3] > s1[3])
        s = s2 if pick2 else s1
        lo, lim = s[0], (s[1] - s[0] + 1) & M32
        sh = max(0, (lim | 1).bit_length() - 7)
        if ((lim + (1 << sh) - 1) >> sh) > 127:
            sh += 1
        pad = (-lim) & ((1 << sh) - 1)
        h = [0] * 256
        for x in u:
            rel = min((ukey(x) - lo) & M32, lim)
            h[(rel + pad) >> sh] += 1

        def apply(s, d, b, c):
            span = lim - 1
            r0 = d << sh
            rlo = r0 - pad if r0 > pad else 0
            rr = ((d + 1) << sh) - 1 - pad
            rhi = min(rr, span)
            s[2] += b
            s[3] = c
            s[0], s[1] = (lo + rlo) & M32, (lo + rhi) & M32
        if shared:
            da, ba, ca = scan(h, r1 - s1[2])
            db, bb, cb = scan(h, r2 - s2[2])
            apply(s2, db, bb, cb)
            apply(s1, da, ba, ca)
        elif pick2:
            apply(s2, *scan(h, r2 - s2[2]))
        else:
            apply(s1, *scan(h, r1 - s1[2]))
        shared = s1[:2] == s2[:2]
    else:
        raise AssertionError('refinement did not converge')
    l1 = s1[0] != s1[1]
    l2 = not shared and s2[0] != s2[1]
    lst, mid = [], 0.0
    if median:
        lo = s1[0] if l1 else s2[0]
        w = ((s2[1] if l2 else s1[1]) - lo + 1) & M32 if (l1 or l2) else 0
        for x in u:
            k = ukey(x)
            if ((k - lo) & M32) < w:
                lst.append(k)
    else:
        A = s1[0] if l1 else (s1[1] + 1) & M32
        w1 = (s1[1] - s1[0] + 1) & M32 if l1 else 0
        wm = 0 if shared else (s2[0] - s1[1] - 1) & M32
        wb = (w1 + wm + (((s2[1] - s2[0] + 1) & M32) if l2 else 0)) & M32
        for x in u:
            k = ukey(x)
            rel = (k - A) & M32
            inm = ((rel - w1) & M32) < wm
            if inm:
                mid += float(np.array([x], np.uint32).view(np.float32)[0])
            if rel < wb and not inm:
                lst.append(k)
    c1off = s1[3] if l1 else 0
    stored = c1off + (s2[3] if l2 else 0)
    assert len(lst) == stored, (len(lst), stored, s1, s2, shared)
    lst.sort()
    rr1, rr2 = r1 - s1[2], r2 - s2[2]
    pb = rr2 if shared else c1off + rr2
    v1 = lst[rr1] if l1 else s1[0]
    v2 = lst[pb] if (l1 if shared else l2) else s2[0]
    if median:
        f = np.float32
        return float((f(key2f(v1)) + f(key2f(v2))) / f(2))
    fixed = 0.0
    if shared:
        lo, hi = (rr1, rr2) if l1 else (0, -1)
        if not l1:
            fixed = key2f(s1[0]) * (rr2 - rr1 + 1)
    else:
        lo = rr1 if l1 else 0
        hi = c1off + rr2 if l2 else c1off - 1
        if not l1:
            fixed += key2f(s1[0]) * (s1[3] - rr1)
        if not l2:
            fixed += key2f(s2[0]) * (rr2 + 1)
    lsum = sum(key2f(lst[i]) for i in range(len(lst)) if lo <= i <= hi)
    return (lsum + fixed + mid) / (n - 2 * kk)


def stress_columns(n):
    """the columns of tests/test_gpu_kernels.py's refinement stress test"""
    rng = np.random.default_rng(100 + n)
    cols = []
    one = np.float32(1.0)
    ulps = np.nextafter(one, np.float32(2)) - one
    c = np.full(n, one, np.float32) + ulps * rng.integers(0, 4, n)
    c[: n // 4] = 3.0
    c[n // 4] = 2.0
    cols.append(c)
    c = np.where(rng.random(n) < 0.5,
                 -5.0 + 1e-6 * rng.standard_normal(n),
                 7.0 + 1e-6 * rng.standard_normal(n)).astype(np.float32)
    cols.append(c)
    c = (1e-3 * rng.standard_normal(n)).astype(np.float32)
    c[0] = 1e30
    cols.append(c)
    c = (rng.standard_normal(n) * 10.0 ** rng.integers(-20, 20, n)).astype(
        np.float32)
    cols.append(c)
    c = np.float32(rng.integers(-2, 3, n)) + np.float32(1e-7) * \
        np.float32(rng.integers(0, 2, n))
    cols.append(c.astype(np.float32))
    c = rng.standard_normal(n).astype(np.float32)
    c[rng.random(n) < 0.1] *= 100.0
    cols.append(c)
    return np.stack(cols, 1).astype(np.float32)


def main():
    n = int(sys.argv[1])
    P = 3001
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, P)).astype(np.float32)
    X[:, 5] = 1.5
    X[:, 6] = np.float32(rng.integers(0, 3, n))
    X[:, 7] = -0.0
    X[: max(1, n // 10), 8] *= 1e30
    X = np.concatenate([X[:, :60], stress_columns(n)], 1)
    for ratio in (0.0, 0.1, 0.2, 0.45):
        k = int(n * ratio)
        if 2 * k >= n:
            continue
        srt = np.sort(X.astype(np.float64), 0)
        for p in range(X.shape[1]):
            got = select(X[:, p], n, k, False)
            want = srt[k:n - k, p].sum() / (n - 2 * k)
            if not abs(got - want) <= 1e-5 * (abs(want) + 1):
                print('trimmed k=%d col %d: got %r want %r' % (k, p, got,
                                                                want))
    for p in range(X.shape[1]):
        got = select(X[:, p], n, 0, True)
        want = float(np.median(X[:, p]).astype(np.float32))
        if got != want:
            print('median col %d: got %r want %r' % (p, got, want))


if __name__ == '__main__':
    main()
