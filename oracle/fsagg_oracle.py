"""TEST INFRASTRUCTURE — numpy restatement of FederatedScope's server-side
aggregation rules (reference v0.3.0, ``federatedscope/core/aggregators``).

This module is the parity checker and the timed CPU baseline ("port") only.
It is never imported by the product package.  Pinned against golden vectors
generated from the real reference (tools/gen_golden.py, tests/golden/).

A "model" is an ``OrderedDict[str, array]``; arrays are numpy arrays of
float32 / float16 / float64 / int64, or :class:`BF16` for bfloat16 keys.
Every rule mirrors the reference's arithmetic op for op:

* elementwise fp32 ops are IEEE-rounded one at a time (numpy never fuses a
  multiply-add), which makes FedAvg / async / online / median bit-exact;
* ATen reductions whose order is ISA-dependent (``torch.dist``, the cascade
  ``sum`` in trimmed mean, ``torch.norm``) are restated with float64
  accumulation and compared under a stated tolerance.
"""
import math
from collections import OrderedDict

import numpy as np

__all__ = [
    'trimmed_group_bound',
    'BF16', 'fedavg_weights', 'para_weighted_avg', 'asyn_weighted_avg',
    'asyn_aggregate', 'online_aggregate', 'krum_distance', 'krum_distance_matrix',
    'krum_scores', 'krum_select', 'krum_aggregate', 'median_update',
    'median_aggregate', 'trimmed_mean_update', 'trimmedmean_aggregate',
    'bulyan_aggregate', 'normbounding_aggregate', 'interpolate_aggregate',
    'add_init', 'f32', 'trimmed_tolerance', 'bulyan_select', 'asyn_weights',
    'FedOptState', 'dequantize', 'ss_fedavg', 'calc_l2_dissim',
    'calc_blocal_dissim', 'b64_tensor',
]

f32 = np.float32


class BF16:
    """bfloat16 array stored as its uint16 bit patterns."""
    __slots__ = ('bits', )

    def __init__(self, bits):
        self.bits = np.asarray(bits, dtype=np.uint16)

    @property
    def shape(self):
        return self.bits.shape

    def to_f32(self):
        return (self.bits.astype(np.uint32) << 16).view(np.float32)

    @staticmethod
    def from_f32(x):
        """Round-to-nearest-even f32 → bf16 (NaN kept quiet)."""
        x = np.asarray(x, dtype=np.float32)
        u = x.view(np.uint32).astype(np.uint64)
        rounded = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
        nan = np.isnan(x)
        if nan.any():
            rounded = np.where(nan, ((u >> 16) | 0x40).astype(np.uint16),
                               rounded)
        return BF16(rounded.astype(np.uint16))


def _kind(a):
    if isinstance(a, BF16):
        return 'bf16'
    return {np.dtype(np.float32): 'f32', np.dtype(np.float16): 'f16',
            np.dtype(np.float64): 'f64'}.get(a.dtype, 'int')


# ---------------------------------------------------------------------------
# FedAvg  (clients_avg_aggregator.py:60-100)
# ---------------------------------------------------------------------------
def fedavg_weights(sizes, ignore_weight=False, use_ss=False):
    """Per-client weights as the reference computes them: Python doubles.

    ``training_set_size`` is a Python sum of the sample sizes (:64-67);
    weight = 1/n if ignore_weight (:77-78), 1.0 under secret sharing (:79-82),
    else size_i / total (:84)."""
    total = 0
    for s in sizes:
        total += s
    n = len(sizes)
    out = []
    for s in sizes:
        if ignore_weight:
            out.append(1.0 / n)
        elif use_ss:
            out.append(1.0)
        else:
            out.append(s / total)
    return out


def _scaled(x, w):
    """``x * w`` with ``w`` a Python float (ATen mul with a wrapped scalar).

    The scalar is read in the op's compute type: float for f32/f16/bf16
    (result rounded to the storage type), double for f64; integer tensors
    promote to the default dtype float32 (x cast first)."""
    k = _kind(x)
    if k == 'f32':
        return x * f32(w)
    if k == 'f16':
        return (x.astype(f32) * f32(w)).astype(np.float16)
    if k == 'bf16':
        return BF16.from_f32(x.to_f32() * f32(w))
    if k == 'f64':
        return x * np.float64(w)
    return x.astype(f32) * f32(w)


def _accum(acc, t):
    """``acc += t`` (in place add, result in acc's dtype)."""
    k = _kind(acc)
    if k == 'bf16':
        tk = t.to_f32() if isinstance(t, BF16) else t.astype(f32)
        return BF16.from_f32(acc.to_f32() + tk)
    if k == 'f16':
        return (acc.astype(f32) + t.astype(f32)).astype(np.float16)
    return (acc + t).astype(acc.dtype)


def para_weighted_avg(models, ignore_weight=False, use_ss=False,
                      recover_fun=None, weights=None):
    """``ClientsAvgAggregator._para_weighted_avg`` (clients_avg_aggregator.py:60-100).

    ``models`` is a list of ``(sample_size, OrderedDict)``.  Keys come from
    client 0; a client missing a key is skipped without renormalising
    (:74-75).  Per element: acc = x0*w0, then acc = acc + xi*wi in list order.
    ``weights`` overrides the per-client weights (used by the async rule)."""
    sizes = [s for s, _ in models]
    total = 0
    for s in sizes:
        total += s
    if weights is None:
        weights = fedavg_weights(sizes, ignore_weight, use_ss)
    out = OrderedDict()
    first = models[0][1]
    for key in first:
        acc = None
        for i, (_, local) in enumerate(models):
            if key not in local:
                continue
            t = _scaled(local[key], weights[i])
            # the reference writes acc at i == 0 (client 0 always has key)
            acc = t if acc is None else _accum(acc, t)
        if use_ss and recover_fun is not None:
            acc = recover_fun(acc)
            acc = np.asarray(acc) / total
            acc = np.asarray(acc, dtype=f32)
        out[key] = acc
    return out


def add_init(init, update):
    """``updated[key] = init[key] + update[key]`` over the update's keys
    (e.g. median_aggregator.py:37-41)."""
    out = OrderedDict()
    for k in update:
        a, b = init[k], update[k]
        if isinstance(a, BF16) or isinstance(b, BF16):
            raise NotImplementedError('bf16 init+update')
        out[k] = (a + b)
    return out


# ---------------------------------------------------------------------------
# Async  (asyn_clients_avg_aggregator.py:14-84)
# ---------------------------------------------------------------------------
def asyn_weights(sizes, staleness, factor, ignore_weight=False):
    total = 0
    for s in sizes:
        total += s
    n = len(sizes)
    out = []
    for i, s in enumerate(sizes):
        w = 1.0 / n if ignore_weight else s / total
        w *= 1.0 / ((1.0 + staleness[i])**factor)  # discount_func :42-51
        out.append(w)
    return out


def asyn_weighted_avg(models, staleness, factor, ignore_weight=False):
    """_para_weighted_avg of the async rule: every key cast with ``.float()``
    (:74-77) and no missing-key check."""
    sizes = [s for s, _ in models]
    w = asyn_weights(sizes, staleness, factor, ignore_weight)
    fl = [(s, OrderedDict((k, _to_float(v)) for k, v in d.items()))
          for s, d in models]
    return para_weighted_avg(fl, weights=w)


def asyn_aggregate(models, staleness, factor, init, ignore_weight=False):
    return add_init(init, asyn_weighted_avg(models, staleness, factor,
                                            ignore_weight))


def _to_float(v):
    if isinstance(v, BF16):
        return v.to_f32()
    return np.asarray(v).astype(f32)


# ---------------------------------------------------------------------------
# Online running mean  (clients_avg_aggregator.py:115-148)
# ---------------------------------------------------------------------------
def _online_mul(t, k):
    """python int k * tensor t (clients_avg_aggregator.py:136-138): the
    tensor's dtype; reduced floats computed in float32 (ATen's opmath) and
    rounded once."""
    t = np.asarray(t)
    if t.dtype == np.int64:
        return t * np.int64(k)
    if t.dtype == np.float16:
        return (t.astype(np.float32) * np.float32(k)).astype(np.float16)
    if t.dtype == np.float64:
        return t * np.float64(k)
    return t.astype(np.float32) * np.float32(k)


_ONLINE_RANK = {np.dtype(np.int64): 0, np.dtype(np.float16): 1,
                np.dtype(np.float32): 2, np.dtype(np.float64): 3}


def _online_add(a, b):
    """tensor + tensor: ATen's promotion (int64 < f16 < f32 < f64), both
    operands cast to the common type, reduced floats added in float32."""
    ct = max(a.dtype, b.dtype, key=lambda d: _ONLINE_RANK[np.dtype(d)])
    if ct == np.float16:
        return (a.astype(np.float16).astype(np.float32) +
                b.astype(np.float16).astype(np.float32)).astype(np.float16)
    return a.astype(ct) + b.astype(ct)


def _online_div(c, d):
    """tensor / python int: integers become float32 (true division)."""
    if c.dtype == np.int64:
        return c.astype(np.float32) / np.float32(d)
    if c.dtype == np.float16:
        return (c.astype(np.float32) / np.float32(d)).astype(np.float16)
    if c.dtype == np.float64:
        return c / np.float64(d)
    return c / np.float32(d)


def online_aggregate(init, clients):
    """reset(): zeros like the server model; inc((s, x)) per client:
    m = (cnt*m + s*x) / (cnt + s) with ATen's dtype rules per op
    (clients_avg_aggregator.py:115-142); cnt += s."""
    m = OrderedDict((k, np.zeros_like(np.asarray(v))) for k, v in
                    init.items())
    cnt = 0
    for s, x in clients:
        for k in m:
            if k not in x:
                continue
            m[k] = _online_div(_online_add(_online_mul(m[k], cnt),
                                           _online_mul(x[k], s)), cnt + s)
        cnt += s
    return m


# ---------------------------------------------------------------------------
# Krum  (krum_aggregator.py:41-90)
# ---------------------------------------------------------------------------
def krum_distance(a, b):
    """Sum over a's keys of the per-key L2 distance (:41-56).  Each per-key
    ``torch.dist`` is restated in float64 and rounded to fp32; the running
    total is an fp32 0-dim tensor started from Python 0.0."""
    dist = f32(0.0)
    for k in a:
        x = _to_float(a[k]).astype(np.float64).ravel()
        y = _to_float(b[k]).astype(np.float64).ravel()
        d = f32(math.sqrt(float(np.dot(x - y, x - y))))
        dist = f32(dist + d)
    return dist


def krum_distance_matrix(paras):
    n = len(paras)
    D = np.zeros((n, n), dtype=f32)
    for a in range(n):
        D[a, a] = np.inf
        for b in range(a + 1, n):
            D[a, b] = D[b, a] = krum_distance(paras[a], paras[b])
    return D


def krum_scores(D, f):
    """Sort each row, sum the first n-f-2 columns with Python slice
    semantics (a non-positive count slices from the end) (:58-77)."""
    n = D.shape[0]
    closest = n - f - 2
    S = np.sort(D, axis=1)[:, :closest]
    return S.astype(np.float64).sum(axis=1).astype(f32)


def krum_select(scores, agg_num):
    order = np.argsort(scores, kind='stable')
    return [int(i) for i in order[:agg_num]]


def krum_aggregate(models, f, agg_num, init, D=None):
    """Multi-Krum: weighted average of the agg_num lowest-score clients in
    ascending-score order, then init + avg (:21-39, :79-90)."""
    if D is None:
        D = krum_distance_matrix([d for _, d in models])
    sel = krum_select(krum_scores(D, f), agg_num)
    avg = para_weighted_avg([models[i] for i in sel])
    return add_init(init, avg), sel


# ---------------------------------------------------------------------------
# Coordinate-wise median  (median_aggregator.py:43-52)
# ---------------------------------------------------------------------------
def median_update(models):
    """(median(T) - median(-T)) / 2 with torch's lower median; NaN if any."""
    first = models[0][1]
    out = OrderedDict()
    for k in first:
        T = np.stack([_to_float(d[k]) for _, d in models], 0)
        n = T.shape[0]
        S = np.sort(T, axis=0)
        lo = S[(n - 1) // 2]
        hi = S[n // 2]
        med_pos = lo                      # torch.median → lower median
        med_neg = -hi                     # lower median of -T is -(upper)
        r = (med_pos - med_neg) / f32(2)
        nan = np.isnan(T).any(axis=0)
        if nan.any():
            r = np.where(nan, np.float32(np.nan), r)
        out[k] = r.astype(f32)
    return out


def median_aggregate(models, init):
    return add_init(init, median_update(models))


# ---------------------------------------------------------------------------
# Trimmed mean  (trimmedmean_aggregator.py:44-57)
# ---------------------------------------------------------------------------
def trimmed_mean_update(models, excluded_num, divisor=None):
    """(Σ all − Σ top-k − Σ bottom-k) / (n − 2k) per coordinate.

    The reference sums ``cat([T, -top, bottom])`` with ATen's cascade sum
    (host-ISA dependent order); here the kept middle is summed in float64 and
    rounded once, then divided in fp32 — compare under tolerance.  Columns
    holding ±inf/NaN reproduce the reference's formula (NaN for k >= 1)."""
    first = models[0][1]
    out = OrderedDict()
    for k in first:
        T = np.stack([_to_float(d[k]) for _, d in models], 0)
        n = T.shape[0]
        S = np.sort(T, axis=0)
        with np.errstate(invalid='ignore'):
            mid = S[excluded_num:n - excluded_num].astype(np.float64).sum(0)
        # Non-finite columns follow the reference's formula literally: with
        # k >= 1 an infinity (or NaN) is both in Σall and among the excluded
        # top/bottom, so Σall − Σtop − Σbottom is inf − inf = NaN; with
        # k == 0 it is Σall itself (±inf, or NaN for NaN / +inf with -inf).
        bad = ~np.isfinite(T).all(0)
        if bad.any():
            has_nan = np.isnan(T).any(0)
            pinf = (T == np.inf).any(0)
            ninf = (T == -np.inf).any(0)
            if excluded_num >= 1:
                nf = np.full(T.shape[1], np.nan)
            else:
                nf = np.where(has_nan | (pinf & ninf), np.nan,
                              np.where(pinf, np.inf, -np.inf))
            mid = np.where(bad, nf, mid)
        div = (n - 2 * excluded_num) if divisor is None else divisor
        out[k] = (mid.astype(f32) / f32(div)).astype(f32)
    return out


def trimmedmean_aggregate(models, ratio, init):
    k = int(len(models) * ratio)
    return add_init(init, trimmed_mean_update(models, k))


def trimmed_tolerance(models, excluded_num, divisor=None):
    """Elementwise abs tolerance: the reference sums n + 2k fp32 values of
    magnitude ≤ max|x| in fp32, so its error is ≤ ~(n+2k)·ε·Σ|x| loosely;
    we use 4·ε·(Σ|x| + 2·Σ|top|)/div, per SURVEY §8c."""
    first = models[0][1]
    out = OrderedDict()
    eps = float(np.finfo(np.float32).eps)
    for k in first:
        T = np.stack([_to_float(d[k]) for _, d in models], 0).astype(
            np.float64)
        n = T.shape[0]
        div = (n - 2 * excluded_num) if divisor is None else divisor
        out[k] = 8 * eps * (2 * np.abs(T).sum(0)) / div + 1e-30
    return out


def trimmed_group_bound(models, excluded_num, divisor=None):
    """Elementwise abs bound on the device trimmed mean against this
    oracle's fp64 middle sum (test infrastructure).  The device
    kernel sums Σ med3(x, L, U) over every value — L the top of the bin
    holding rank k, U the bottom of the bin holding rank n − k − 1, so each
    term is |x| of a kept value or at most max(|L|, |U|) — in fp32 groups
    of at most 12 terms widened to fp64, then removes L·#(≤ L) + U·#(≥ U)
    exactly: its sum is off by at most 11·u·Σ|terms| (u = 2^-24).  |L| and
    |U| are at most 1.125·max(|x_(k)|, |x_(n−k−1)|) (a bin spans 1/8 octave)
    or, for the bin of magnitudes below the digit base, |x|max·2^-15.
    Divided by the divisor; the final cast, division and init add round
    once each and are covered by the callers' ε·|result| terms.  Far inside
    the reference's own bound (:func:`trimmed_tolerance`, 16ε·Σ|x|/div)."""
    first = models[0][1]
    out = OrderedDict()
    u = 2.0 ** -24
    for k in first:
        T = np.sort(np.stack([_to_float(d[k]) for _, d in models], 0).astype(
            np.float64), 0)
        n = T.shape[0]
        div = (n - 2 * excluded_num) if divisor is None else divisor
        F = np.where(np.isfinite(T), T, 0.0)
        kept = np.abs(F[excluded_num:n - excluded_num]).sum(0)
        edge = np.maximum(np.abs(F[excluded_num]),
                          np.abs(F[n - excluded_num - 1]))
        amax = np.abs(F).max(0)
        out[k] = 11 * u * (kept + n * (1.125 * edge + amax * 2.0 ** -15)) / div
    return out


# ---------------------------------------------------------------------------
# Bulyan  (bulyan_aggregator.py:75-106)
# ---------------------------------------------------------------------------
def bulyan_select(models, f, rate, D=None):
    if D is None:
        D = krum_distance_matrix([d for _, d in models])
    scores = krum_scores(D, f)
    order = np.argsort(scores, kind='stable')
    keep = len(models) - int(2 * rate * f)
    return [int(i) for i in order[:max(keep, 0)]], scores


def bulyan_aggregate(models, f, rate, init, D=None):
    sel, _ = bulyan_select(models, f, rate, D)
    reliable = [models[i] for i in sel]
    k = int(rate * f)
    gamma = len(reliable) - 2 * k
    upd = trimmed_mean_update(reliable, k, divisor=gamma)
    # keys follow client 0 of the ORIGINAL list (global_update deepcopy, :81)
    upd = OrderedDict((key, upd[key]) for key in models[0][1])
    return add_init(init, upd), sel


# ---------------------------------------------------------------------------
# Norm bounding  (normbounding_aggregator.py:35-70)
# ---------------------------------------------------------------------------
def normbounding_aggregate(models, bound, init):
    tmp = []
    for s, d in models:
        present = [k for k in init if k in d]
        flat = np.concatenate([_to_float(d[k]).ravel() for k in present])
        norm = f32(math.sqrt(float(np.dot(flat.astype(np.float64),
                                          flat.astype(np.float64)))))
        if norm > bound:
            # bound / torch.norm(...): Tensor.__rtruediv__ = reciprocal()·other
            rate = f32(f32(f32(1.0) / norm) * f32(bound))
            scaled = rate * flat
            rec = OrderedDict()
            off = 0
            for k in init:
                if k in present:
                    sz = int(np.prod(init[k].shape))
                    rec[k] = scaled[off:off + sz].reshape(init[k].shape)
                    off += sz
                else:
                    rec[k] = init[k].copy()
            tmp.append((s, rec))
        else:
            tmp.append((s, d))
    return add_init(init, para_weighted_avg(tmp))


# ---------------------------------------------------------------------------
# Server/clients interpolation  (server_clients_interpolate_aggregator.py:20-30)
# ---------------------------------------------------------------------------
def interpolate_aggregate(models, global_model, beta):
    avg = para_weighted_avg(models)
    return para_weighted_avg([((1 - beta), global_model), (beta, avg)])


# ---------------------------------------------------------------------------
# FedOpt  (fedopt_aggregator.py:26-44 + torch.optim single-tensor steps)
# ---------------------------------------------------------------------------
def _fma32(a, b, c):
    """fp32 fused multiply-add, emulated in float64 (a·b is exact there)."""
    return (np.float64(a) * np.float64(b) + np.asarray(c, np.float64)).astype(
        f32)


class FedOptState:
    """Server optimizer state carried across rounds (torch.optim
    single-tensor semantics — SGD, Adam, AdamW, Adagrad, RMSprop — with
    ATen's vectorised fmadd for add(alpha) and lerp; tolerance-pinned).
    float32 parameters use an exact fp32 fma; float64 ones plain float64 ops
    (numpy has no fma: a few ulps apart, within the float64 tolerance).
    Follows torch/optim/{sgd,adam,adagrad,rmsprop}.py _single_tensor_*."""

    def __init__(self, params, opt):
        first = np.asarray(next(iter(params.values())))
        self.dt = np.float64 if first.dtype == np.float64 else f32
        self.params = OrderedDict((k, np.asarray(v, self.dt).copy())
                                  for k, v in params.items())
        self.opt = dict(opt)
        self.buf = {}
        self.m = {}
        self.v = {}
        self.vmax = {}
        self.ga = {}
        self.steps = {}

    def _fma(self, a, b, c):
        if self.dt == f32:
            return _fma32(a, b, c)
        return np.float64(a) * np.float64(b) + np.asarray(c, np.float64)

    def _lerp(self, a, b, w):
        """torch.lerp(a, b, w) on CPU (w < 0.5: a + w·(b − a) as an fma)."""
        T = self.dt
        if w < 0.5:
            return self._fma(T(w), b - a, a)
        return b - (b - a) * T(1 - w)

    def step(self, models):
        avg = para_weighted_avg(models)
        o = self.opt
        T = self.dt
        typ = o['type']
        for k, x in self.params.items():
            if k not in avg:
                continue
            t = self.steps[k] = self.steps.get(k, 0) + 1
            g = x - avg[k]
            if o.get('maximize', False):
                g = -g
            wd = o.get('weight_decay', 1e-2 if typ == 'AdamW' else 0.0)
            decoupled = typ == 'AdamW'
            if wd and not decoupled:
                g = self._fma(x, T(wd), g)
            if typ == 'SGD':
                mom = o.get('momentum', 0.0)
                if mom:
                    if k not in self.buf:
                        self.buf[k] = g.copy()
                    else:
                        self.buf[k] = self._fma(
                            g, T(1 - o.get('dampening', 0.0)),
                            self.buf[k] * T(mom))
                    g = self._fma(self.buf[k], T(mom), g) if o.get(
                        'nesterov', False) else self.buf[k]
                self.params[k] = self._fma(g, T(-o['lr']), x)
            elif typ in ('Adam', 'AdamW'):
                if wd and decoupled:
                    x = x * T(1 - o['lr'] * wd)
                b1, b2 = o.get('betas', (0.9, 0.999))
                eps = o.get('eps', 1e-8)
                m = self.m.get(k, np.zeros_like(x))
                v = self.v.get(k, np.zeros_like(x))
                m = self._lerp(m, g, 1 - b1)
                v = v * T(b2) + (T(1 - b2) * g) * g
                bc1 = 1 - b1**t
                bc2 = 1 - b2**t
                vd = v
                if o.get('amsgrad', False):
                    vd = np.maximum(self.vmax.get(k, np.zeros_like(x)), v)
                    self.vmax[k] = vd
                denom = np.sqrt(vd) / T(bc2**0.5) + T(eps)
                self.params[k] = x + (T(-(o['lr'] / bc1)) * m) / denom
                self.m[k], self.v[k] = m, v
            elif typ == 'Adagrad':
                ss = self.v.get(k, np.full_like(
                    x, o.get('initial_accumulator_value', 0.0)))
                ss = ss + g * g
                self.v[k] = ss
                clr = o['lr'] / (1 + (t - 1) * o.get('lr_decay', 0.0))
                std = np.sqrt(ss) + T(o.get('eps', 1e-10))
                self.params[k] = x + (T(-clr) * g) / std
            elif typ == 'RMSprop':
                alpha = o.get('alpha', 0.99)
                eps = o.get('eps', 1e-8)
                mom = o.get('momentum', 0.0)
                v = self.v.get(k, np.zeros_like(x)) * T(alpha)
                v = v + (T(1 - alpha) * g) * g
                self.v[k] = v
                if o.get('centered', False):
                    ga = self._lerp(self.ga.get(k, np.zeros_like(x)), g,
                                    1 - alpha)
                    self.ga[k] = ga
                    d = np.sqrt(v + (T(-1) * ga) * ga)
                else:
                    d = np.sqrt(v)
                d = d + T(eps)
                if mom > 0:
                    b = self.buf.get(k, np.zeros_like(x)) * T(mom)
                    b = b + g / d
                    self.buf[k] = b
                    self.params[k] = self._fma(b, T(-o['lr']), x)
                else:
                    self.params[k] = x + (T(-o['lr']) * g) / d
            else:
                raise NotImplementedError(typ)
        return OrderedDict((k, v.copy()) for k, v in self.params.items())


# ---------------------------------------------------------------------------
# §8(f) rows: wire formats, secret sharing, update-dissimilarity metrics
# ---------------------------------------------------------------------------
def dequantize(wire):
    """compression/utils.py:64-90: ``x.weight_quant * x.weight_scale`` in
    fp32 (int codes promoted to float32, times the fp32 scale, one rounding),
    other keys passed through, ``*.weight_scale`` dropped."""
    out = OrderedDict()
    for key, value in wire.items():
        if 'weight_quant' in key:
            alpha = np.float32(np.asarray(
                wire[key.replace('weight_quant', 'weight_scale')]))
            out[key.replace('weight_quant', 'weight')] = \
                np.asarray(value).astype(np.float32) * alpha
        elif 'weight_scale' in key:
            continue
        else:
            out[key] = value
    return out


def _py_mod(a, b):
    """numpy's float64 remainder (the sign of the divisor)."""
    m = np.fmod(a, b)
    fix = (m != 0) & ((b < 0) != (m < 0))
    m = np.where(fix, m + b, m)
    return np.where(m == 0, np.copysign(0.0, b), m)


def ss_fedavg(models, mod_number, maximum, epsilon, ignore_weight=False):
    """clients_avg_aggregator.py:79-98 with AdditiveSecretSharing
    .fixedpoint2float (secret_sharing.py:93-98): Σ shares·w (float64, list
    order; w = 1.0, or 1/n with ignore_weight, which the reference tests
    first, :77-82), x %= mod, x > maximum ? -(mod - x)/eps : x/eps,
    ÷ total sample size, → fp32."""
    total = 0
    for s, _ in models:
        total += s
    w = 1.0 / len(models) if ignore_weight else 1.0
    mod = np.float64(float(mod_number))
    mx = np.float64(float(maximum))
    eps = np.float64(epsilon)
    out = OrderedDict()
    for key in models[0][1]:
        acc = None
        for _, m in models:
            if key not in m:
                continue
            x = np.asarray(m[key]).astype(np.float64) * w
            acc = x if acc is None else acc + x
        x = _py_mod(acc, mod)
        r = np.where(x > mx, -1 * (mod - x) / eps, x / eps)
        out[key] = (r / np.float64(total)).astype(np.float32)
    return out


def calc_l2_dissim(last, models):
    """metric_calculator.py:360-372, fp64 accumulation (the reference's fp32
    torch.norm is ISA-dependent; compared under a tolerance)."""
    raw = []
    for _, m in models:
        sq = 0.0
        for k, w in m.items():
            g = (np.asarray(w, np.float32) - np.asarray(last[k], np.float32))
            sq += float(np.sum(g.astype(np.float64) ** 2))
        raw.append(math.sqrt(sq))
    return {'raw': raw, 'mean': float(np.mean(raw))}


def calc_blocal_dissim(last, models):
    """metric_calculator.py:309-357 with fp64 sums of squares; the global
    update Σ_i fl32(w_i · g_i) keeps the reference's fp32 op order."""
    w = np.asarray([s for s, _ in models], dtype=np.float64)
    w = w / np.sum(w)
    out = OrderedDict()
    for k in models[0][1]:
        avg = 0.0
        glob = np.zeros(np.asarray(last[k]).shape, np.float32)
        for i, (_, m) in enumerate(models):
            g = np.asarray(m[k], np.float32) - np.asarray(last[k], np.float32)
            avg += w[i] * float(np.sum(g.astype(np.float64) ** 2))
            glob = glob + np.float32(w[i]) * g
        out[k] = math.sqrt(avg / float(np.sum(glob.astype(np.float64) ** 2)))
    return out


# ---------------------------------------------------------------------------
# gRPC uploads: base64(pickle(tensor))
# ---------------------------------------------------------------------------
_B64_STORAGE = {'FloatStorage': np.float32, 'DoubleStorage': np.float64,
                'HalfStorage': np.float16, 'LongStorage': np.int64,
                'IntStorage': np.int32, 'ShortStorage': np.int16,
                'CharStorage': np.int8, 'ByteStorage': np.uint8,
                'BoolStorage': np.bool_, 'BFloat16Storage': 'bf16'}


def _pickle_ops(buf, pos=0):
    """(ops, end) of the pickle starting at ``buf[pos:]`` — the stdlib
    disassembler, which only reads opcodes and executes nothing."""
    import pickletools
    ops = list(pickletools.genops(buf[pos:]))
    return ops, pos + ops[-1][2] + 1


def b64_tensor(text):
    """The tensor a b64serializer payload carries (message.py:8-9:
    ``base64.b64encode(pickle.dumps(x))``; decoded by param2tensor,
    utils.py:95-105), restated with the stdlib: base64-decode everything,
    disassemble the outer pickle (torch's ``_rebuild_tensor_v2(
    _load_from_bytes(payload), offset, size, stride, requires_grad, {})``)
    and the legacy torch.save stream in the payload (magic, protocol,
    sys_info, the ('storage', torch.<T>Storage, key, location, numel)
    persistent id, [key], then numel as 8 LE bytes + raw elements).
    Returns a contiguous numpy array (BF16 for bfloat16)."""
    import base64
    raw = base64.b64decode(text, validate=True)
    ops, end = _pickle_ops(raw)
    assert end == len(raw)
    names = [op.name for op, _, _ in ops]
    ib = next(i for i, n in enumerate(names)
              if n in ('BINBYTES', 'SHORT_BINBYTES', 'BINBYTES8'))
    payload = ops[ib][1]
    # after the storage's REDUCE: offset, size tuple, stride tuple, bool
    ir = names.index('REDUCE', ib)
    stack = []
    for op, arg, _ in ops[ir + 1:]:
        n = op.name
        if n in ('BININT', 'BININT1', 'BININT2', 'LONG1'):
            stack.append(int(arg))
        elif n == 'MARK':
            stack.append('mark')
        elif n in ('TUPLE1', 'TUPLE2', 'TUPLE3'):
            k = int(n[-1])
            t = tuple(stack[-k:])
            del stack[-k:]
            stack.append(t)
        elif n == 'EMPTY_TUPLE':
            stack.append(())
        elif n == 'TUPLE':
            m = len(stack) - 1 - stack[::-1].index('mark')
            t = tuple(stack[m + 1:])
            del stack[m:]
            stack.append(t)
        elif n in ('NEWFALSE', 'NEWTRUE'):
            stack.append(n == 'NEWTRUE')
            break
    offset, size, stride, _ = stack[-4:]
    # the legacy stream: five pickles, then numel + the raw storage
    pos = 0
    cls = None
    for j in range(5):
        pops, pos = _pickle_ops(payload, pos)
        if j == 3:
            cls = next(arg for op, arg, _ in pops if op.name == 'GLOBAL')
    numel = int.from_bytes(payload[pos:pos + 8], 'little')
    dt = _B64_STORAGE[cls.split()[1]]
    if dt == 'bf16':
        store = np.frombuffer(payload[pos + 8:], dtype=np.uint16)
    else:
        store = np.frombuffer(payload[pos + 8:], dtype=dt)
    assert store.size == numel
    es = store.itemsize
    view = np.lib.stride_tricks.as_strided(
        store[offset:], shape=size, strides=tuple(es * s for s in stride))
    out = np.array(view)
    return BF16(out) if dt == 'bf16' else out
