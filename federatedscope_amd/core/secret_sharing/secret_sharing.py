"""Server side of additive secret sharing (federatedscope/core/
secret_sharing/secret_sharing.py).

Splitting happens on the CLIENTS (Client.callback_funcs_for_model_para,
client.py:374-400, with the reference's AdditiveSecretSharing) and is not
rebuilt here.  The SERVER side — Σ shares, fixedpoint2float, ÷ total — is
the aggregation hot path and runs fused on the GPU (fsagg_ss_recover_f32,
called by ClientsAvgAggregator when cfg.federate.use_ss); :func:`ss_params`
reads the constants of the recover function the server is handed.
"""


def ss_params(recover_fun):
    """(mod, maximum, epsilon) as doubles for the device recovery.

    ``recover_fun`` is what the reference's server passes as agg_info's
    ``recover_fun``: ``AdditiveSecretSharing(...).fixedpoint2float``, an
    ``np.vectorize`` of the bound ``_fixedpoint2float`` (secret_sharing.py:
    88-98) — its owner holds ``mod_number``, ``maximum`` and ``epsilon``.
    Any callable that carries those three attributes itself (or whose
    ``__self__`` does) is accepted too.  Other recover functions have no
    device path and raise."""
    for cand in (getattr(getattr(recover_fun, 'pyfunc', None), '__self__',
                         None),
                 getattr(recover_fun, '__self__', None), recover_fun):
        if cand is not None and all(hasattr(cand, a) for a in
                                    ('mod_number', 'maximum', 'epsilon')):
            # numpy converts the Python ints to float64 in `x % mod_number`
            # and `mod_number - x` (2·2^60 + 1 rounds to 2^61)
            return (float(cand.mod_number), float(cand.maximum),
                    float(cand.epsilon))
    raise NotImplementedError(
        'device secret-sharing recovery needs the fixed-point constants '
        '(mod_number, maximum, epsilon) of AdditiveSecretSharing; got %r' %
        recover_fun)
