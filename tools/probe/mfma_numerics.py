#!/usr/bin/env python3
"""How gfx950's v_mfma_f32_16x16x32_bf16 rounds, and the error of
pairgram.hip's k-step (tools only, never in the product).

raw:   one MFMA, D = C + Σ_k A[i][k]·B[k][j] on bf16 inputs chosen to expose
       the accumulation (exact products? one rounding or many? to nearest or
       toward zero? does alignment to the largest term drop small ones?).
       Every output is compared with the exact sum (math.fsum of the exact
       fp64 products plus the exact residual) rounded to fp32.
kstep: the product's k-step (three bf16 limbs, six chained MFMAs) on fp32
       rows of several data families: error / (u · Σ|x_a·x_b|), u = 2^-24.

Writes one JSON object per family to stdout."""
import ctypes
import json
import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
U = 2.0 ** -24


def lib():
    so = os.path.join(HERE, 'bin', 'libmfma_numerics.so')
    L = ctypes.CDLL(so)
    for f in (L.probe_mfma_raw, L.probe_mfma_kstep):
        f.restype = ctypes.c_int
    return L


def bf16_bits(x):
    """fp32 array → bf16 bits, round to nearest even (the values chosen are
    exactly representable, this only truncates the zero low half)."""
    b = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    r = ((b >> 16) & 1) + 0x7fff
    return ((b + r) >> 16).astype(np.uint16)


def bf16_val(bits):
    return (bits.astype(np.uint32) << 16).view(np.float32)


def rand_bf16(rng, shape, emin, emax):
    m = rng.integers(128, 256, size=shape).astype(np.float64) / 128.0
    e = rng.integers(emin, emax + 1, size=shape)
    s = np.where(rng.random(shape) < 0.5, -1.0, 1.0)
    return (s * m * np.exp2(e)).astype(np.float32)


def raw_cases(fam, rng, nc):
    A = np.zeros((nc, 16, 32), np.float32)
    B = np.zeros((nc, 32, 16), np.float32)
    C = np.zeros((nc, 16, 16), np.float32)
    if fam == 'int':           # small integers: every sum exact (mapping)
        A[:] = rng.integers(-8, 9, A.shape)
        B[:] = rng.integers(-8, 9, B.shape)
        C[:] = rng.integers(-64, 65, C.shape)
    elif fam == 'wide':        # exponents over 2^±20, random signs
        A[:] = rand_bf16(rng, A.shape, -10, 10)
        B[:] = rand_bf16(rng, B.shape, -10, 10)
        C[:] = rand_bf16(rng, C.shape, -20, 20)
    elif fam == 'one_plus_tiny':   # 1 + 31 same-sign terms < half an ulp
        A[:, :, 0] = 1.0
        B[:, 0, :] = 1.0
        A[:, :, 1:] = 2.0 ** -13
        B[:, 1:, :] = rand_bf16(rng, (nc, 31, 16), -14, -12).__abs__()
    elif fam == 'cancel':      # +X and −X, then small terms
        A[:, :, 0] = 2.0 ** 10
        A[:, :, 1] = 2.0 ** 10
        B[:, 0, :] = 2.0 ** 10
        B[:, 1, :] = -2.0 ** 10
        A[:, :, 2:] = rand_bf16(rng, (nc, 16, 30), -12, -8)
        B[:, 2:, :] = rand_bf16(rng, (nc, 30, 16), -12, -8)
    elif fam == 'c_dominant':  # |C| ≫ the products
        A[:] = rand_bf16(rng, A.shape, -2, 2)
        B[:] = rand_bf16(rng, B.shape, -2, 2)
        C[:] = rand_bf16(rng, C.shape, 18, 22)
    elif fam == 'ties':        # C = 1, products sum to 1, 2 or 3 half-ulps
        C[:] = 1.0
        A[:, :, 0] = 2.0 ** -12
        t = rng.integers(1, 4, size=(nc, 16))
        B[:, 0, :] = t * 2.0 ** -12
    elif fam.startswith('window'):      # 1 + 31 terms of ±1.99·2^-k
        # window<k>[n]: the alignment window below the largest term
        neg = fam.endswith('n')
        k = int(fam[6:].rstrip('n'))
        A[:, :, 0] = 1.0
        B[:, 0, :] = 1.0
        A[:, :, 1:] = 2.0 ** -12
        B[:, 1:, :] = (-1.0 if neg else 1.0) * 1.9921875 * 2.0 ** (12 - k)
    elif fam == 'mixed_sign_same_mag':   # Σ of ±1·(1+m) terms, cancellation
        A[:] = rand_bf16(rng, A.shape, 0, 0)
        B[:] = rand_bf16(rng, B.shape, 0, 0)
        C[:] = rand_bf16(rng, C.shape, -30, -20)
    return A, B, C


def exact_sum(terms):
    s = math.fsum(terms)
    r = math.fsum(terms + [-s])
    return s, r


def round32(s, r, mode):
    """fp32 rounding of the exact value s + r (|r| ≤ half an fp64 ulp)."""
    f = np.float32(s)
    fd = float(f)
    if mode == 'rne':
        if fd != s:
            # s at an fp32 midpoint: the residual decides
            lo = float(np.nextafter(f, np.float32(-np.inf)))
            hi = float(np.nextafter(f, np.float32(np.inf)))
            for nb in (lo, hi):
                if (nb + fd) / 2 == s and r != 0.0:
                    want_up = r > 0
                    return max(fd, nb) if want_up else min(fd, nb)
        return fd
    # rtz: the largest magnitude ≤ |exact|
    d = math.fsum([fd, -s, -r])
    if fd != 0.0 and (d > 0) == (fd > 0) and d != 0.0:
        return float(np.nextafter(f, np.float32(0.0)))
    return fd


def ulp32(v):
    v = abs(v)
    if v < 2.0 ** -126:
        return 2.0 ** -149
    return 2.0 ** (math.floor(math.log2(v)) - 23)


def run_raw(L, fam, nc=256, seed=0):
    rng = np.random.default_rng(seed)
    A, B, C = raw_cases(fam, rng, nc)
    ab, bb = bf16_bits(A), bf16_bits(B)
    A, B = bf16_val(ab).reshape(A.shape), bf16_val(bb).reshape(B.shape)
    dA = torch.from_numpy(ab.view(np.int16)).cuda()
    dB = torch.from_numpy(bb.view(np.int16)).cuda()
    dC = torch.from_numpy(C).cuda()
    dD = torch.empty_like(dC)
    assert L.probe_mfma_raw(ctypes.c_void_p(dA.data_ptr()),
                            ctypes.c_void_p(dB.data_ptr()),
                            ctypes.c_void_p(dC.data_ptr()),
                            ctypes.c_void_p(dD.data_ptr()), nc) == 0
    D = dD.cpu().numpy()
    P = A.astype(np.float64)[:, :, None, :] * \
        B.astype(np.float64).transpose(0, 2, 1)[:, None, :, :]
    n_rne = n_rtz = n = 0
    worst_ulp = worst_rel = worst_max = 0.0
    for c in range(nc):
        for i in range(16):
            for j in range(16):
                t = P[c, i, j].tolist() + [float(C[c, i, j])]
                s, r = exact_sum(t)
                got = float(D[c, i, j])
                n += 1
                n_rne += got == round32(s, r, 'rne')
                n_rtz += got == round32(s, r, 'rtz')
                e = abs(math.fsum([got, -s, -r]))
                worst_ulp = max(worst_ulp, e / ulp32(s + r))
                tot = math.fsum(abs(x) for x in t)
                if tot > 0:
                    worst_rel = max(worst_rel, e / (U * tot))
                    worst_max = max(worst_max, e / (U * max(abs(x)
                                                             for x in t)))
    return {'probe': 'raw', 'family': fam, 'outputs': n,
            'max_err_over_u_max_abs_term': worst_max,
            'frac_equal_rne_of_exact': n_rne / n,
            'frac_equal_rtz_of_exact': n_rtz / n,
            'max_err_ulps_of_result': worst_ulp,
            'max_err_over_u_sum_abs_terms': worst_rel}


def kstep_rows(fam, rng, nc):
    sh = (nc, 16, 32)
    if fam == 'gaussian':
        return rng.standard_normal(sh), rng.standard_normal(sh)
    if fam == 'int8_grid':
        s = 0.37 / 127
        return (rng.integers(-127, 128, sh) * s, rng.integers(-127, 128, sh)
                * s)
    if fam == 'student_t3':
        return rng.standard_t(3, sh), rng.standard_t(3, sh)
    if fam == 'offset':           # both rows = common offset + small noise
        off = 0.5 + rng.standard_normal((nc, 1, 32)) * 0.0
        return (off + 1e-3 * rng.standard_normal(sh),
                off + 1e-3 * rng.standard_normal(sh))
    if fam == 'sparse':
        a, b = rng.standard_normal(sh), rng.standard_normal(sh)
        a[rng.random(sh) < 0.5] = 0
        b[rng.random(sh) < 0.5] = 0
        return a, b
    if fam == 'wide_exp':
        return (rand_bf16(rng, sh, -30, 30) * (1 + rng.random(sh)),
                rand_bf16(rng, sh, -30, 30) * (1 + rng.random(sh)))
    if fam == 'same_row':         # G_aa: every product positive
        a = rng.standard_normal(sh)
        return a, a
    raise ValueError(fam)


def run_kstep(L, fam, nc=256, seed=1):
    rng = np.random.default_rng(seed)
    XA, XB = (np.ascontiguousarray(x, dtype=np.float32)
              for x in kstep_rows(fam, rng, nc))
    dA, dB = torch.from_numpy(XA).cuda(), torch.from_numpy(XB).cuda()
    dG = torch.empty((nc, 16, 16), dtype=torch.float32, device='cuda')
    assert L.probe_mfma_kstep(ctypes.c_void_p(dA.data_ptr()),
                              ctypes.c_void_p(dB.data_ptr()),
                              ctypes.c_void_p(dG.data_ptr()), nc) == 0
    G = dG.cpu().numpy()
    P = XA.astype(np.float64)[:, :, None, :] * \
        XB.astype(np.float64)[:, None, :, :]
    worst = worst_res = 0.0
    errs = []
    for c in range(nc):
        for i in range(16):
            for j in range(16):
                t = P[c, i, j].tolist()
                s, r = exact_sum(t)
                e = abs(math.fsum([float(G[c, i, j]), -s, -r]))
                tot = math.fsum(abs(x) for x in t)
                if tot > 0:
                    q = e / (U * tot)
                    errs.append(q)
                    worst = max(worst, q)
                if s != 0:
                    worst_res = max(worst_res, e / (U * abs(s + r)))
    errs = np.array(errs)
    return {'probe': 'kstep', 'family': fam, 'outputs': int(errs.size),
            'max_err_over_u_sum_abs_products': worst,
            'p999_err_over_u_sum_abs_products': float(np.quantile(errs,
                                                                  0.999)),
            'mean_err_over_u_sum_abs_products': float(errs.mean()),
            'max_err_over_u_result': worst_res}


def main():
    L = lib()
    which = sys.argv[1:] or ['raw', 'kstep']
    if 'window' in which:
        which = ['raw', 'window']
    if 'raw' in which:
        fams = ['int', 'wide', 'one_plus_tiny', 'cancel', 'c_dominant',
                'ties', 'mixed_sign_same_mag']
        if 'window' in which:
            fams = ['window%d%s' % (k, sg) for k in range(22, 33)
                    for sg in ('', 'n')]
        for fam in fams:
            print(json.dumps(run_raw(L, fam, nc=16 if fam.startswith(
                'window') else 256)), flush=True)
    if 'kstep' in which:
        for fam in ('gaussian', 'int8_grid', 'student_t3', 'offset',
                    'sparse', 'wide_exp', 'same_row'):
            print(json.dumps(run_kstep(L, fam)), flush=True)


if __name__ == '__main__':
    main()
