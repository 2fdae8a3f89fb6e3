"""CPU checks of the order-statistic select kernel's index arithmetic,
through its lane-level Python model (tools/sim_select.py): octave digits and
their key intervals, the interval refinement plans, the band compaction and
the list positions must give exactly numpy's order statistics — median
bit-exact, trimmed mean to fp64 rounding — on random, tied, signed-zero,
huge-outlier and ulp-cluster columns.  (The GPU tests check the kernel
itself against the oracle and the reference goldens.)"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))), 'tools'))
import sim_select as S  # noqa: E402


def columns(n, rng):
    cols = [rng.standard_normal(n).astype(np.float32) for _ in range(4)]
    c = rng.standard_normal(n).astype(np.float32)
    c[rng.random(n) < 0.1] *= 100.0
    cols.append(c)                                   # C5-like outliers
    cols.append(np.full(n, 1.5, np.float32))         # all tied
    cols.append(np.float32(rng.integers(0, 3, n)))   # heavy ties, zeros
    c = np.zeros(n, np.float32)
    c[: n // 2] = -0.0
    cols.append(c)                                   # signed zeros
    c = (1e-3 * rng.standard_normal(n)).astype(np.float32)
    c[:3] = [1e30, -1e30, 3e29]
    cols.append(c)                                   # > 16 octaves: refine
    return np.stack(cols + list(S.stress_columns(n).T), 1)


@pytest.mark.parametrize('n', [65, 100, 200, 255])
def test_select_model_matches_numpy(n):
    rng = np.random.default_rng(n)
    X = columns(n, rng)
    f = np.float32
    for p in range(X.shape[1]):
        col = X[:, p]
        s = np.sort(col)
        want = float((f(s[(n - 1) // 2]) + f(s[n // 2])) / f(2))
        got = S.select(col, n, 0, True)
        assert got == want or (got == 0.0 and want == 0.0), (n, p, got,
                                                            want)
        for ratio in (0.0, 0.2, 0.45):
            k = int(n * ratio)
            ref = np.sort(col.astype(np.float64))[k:n - k].sum() / (n - 2 * k)
            got = S.select(col, n, k, False)
            tol = 1e-12 * (np.abs(col.astype(np.float64)).sum() + 1.0)
            assert abs(got - ref) <= tol, (n, p, k, got, ref)
