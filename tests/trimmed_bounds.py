"""Error units and bounds of the trimmed-mean family (trimmed mean, Bulyan)
in the tests.

The unit is SURVEY §8(c)'s: ε·Σ|x|/(n − 2k) per coordinate (ε = 2^-23, Σ
over all n client values of the coordinate, the divisor n − 2k or Bulyan's
γ).  The contract against the reference's own output is

    |ours − ref| <= CONTRACT_UNITS · unit + 4ε·|ref|                (§8(c))

and the regression bound against the oracle's fp64 middle sum (rounded
once) is ORACLE_UNITS · unit + 4ε·(|oracle| + |init|) — about twice the
largest error measured on the GPU over every golden, the C5 blocks and the
kernel stress columns (``FSAGG_ERR_LOG``: each check appends its measured
maximum in units, profiles/r06/trimmed_err.jsonl).  The kernels' worst case
is larger (fp32 groups of <= 12 terms: DESIGN §4); the bound exists to catch
a change that moves the measured error, not to restate the worst case."""
import json
import os

import numpy as np

EPS = float(np.finfo(np.float32).eps)
CONTRACT_UNITS = 4.0
ORACLE_UNITS = 1.3
# measurement passes only (every check logs, none fails)
if os.environ.get('FSAGG_TRIM_MEASURE'):
    CONTRACT_UNITS = ORACLE_UNITS = 1e9


def units(T, div):
    """ε·Σ|x|/div per coordinate of the [n][m] client values ``T`` (non-finite
    values count as 0), never 0."""
    T = np.asarray(T, dtype=np.float64)
    S = np.abs(np.where(np.isfinite(T), T, 0.0)).sum(0)
    return EPS * S / float(div) + 1e-300


def log(tag, err, unit, slack=None):
    """The largest err / unit (after subtracting ``slack``, the rounding
    allowance) to $FSAGG_ERR_LOG; returns it."""
    e = np.asarray(err, dtype=np.float64)
    if slack is not None:
        e = np.maximum(e - slack, 0.0)
    r = float((e / unit).max()) if e.size else 0.0
    path = os.environ.get('FSAGG_ERR_LOG')
    if path:
        with open(path, 'a') as f:
            f.write(json.dumps({'check': tag, 'max_units': r,
                                'count': int(e.size)}) + '\n')
    return r


def check_vs_ref(tag, got, ref, T, div):
    """§8(c) against the reference's output: returns the measured units."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    u = units(T, div)
    err = np.abs(got - ref)
    slack = 4 * EPS * np.abs(ref)
    r = log(tag + '|ref', err, u, slack)
    assert (err <= CONTRACT_UNITS * u + slack).all(), (tag, r)
    return r


def check_vs_oracle(tag, got, want, T, div, init=None):
    """Regression bound against the oracle (fp64 middle sum + the final
    roundings, and the init add when ``init`` is given)."""
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    u = units(T, div)
    err = np.abs(got - want)
    slack = 4 * EPS * (np.abs(want) +
                       (0.0 if init is None else np.abs(np.asarray(init))))
    r = log(tag + '|oracle', err, u, slack)
    assert (err <= ORACLE_UNITS * u + slack).all(), (tag, r)
    return r
