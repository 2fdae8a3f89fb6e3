"""Additive secret sharing (drop-in for
federatedscope/core/secret_sharing/secret_sharing.py).

Splitting happens on the CLIENTS (Client.callback_funcs_for_model_para,
client.py:374-400) and stays host numpy here, with the reference's exact
semantics (np.vectorize'd fixed-point maps, int64 random frames, a float64
last frame).  The SERVER side — Σ shares, fixedpoint2float, ÷ total — is the
aggregation hot path and runs fused on the GPU (fsagg_ss_recover_f32, called
by ClientsAvgAggregator when cfg.federate.use_ss); :func:`ss_params` tells
it the constants of a recover function.
"""
from abc import ABC, abstractmethod

import numpy as np

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


class SecretSharing(ABC):
    def __init__(self):
        pass

    @abstractmethod
    def secret_split(self, secret):
        pass

    @abstractmethod
    def secret_reconstruct(self, secret_seq):
        pass


class AdditiveSecretSharing(SecretSharing):
    """Fixed point with ``epsilon`` = 1e8 steps modulo 2·2^size + 1
    (secret_sharing.py:22-98)."""

    def __init__(self, shared_party_num, size=60):
        super(SecretSharing, self).__init__()
        assert shared_party_num > 1, "AdditiveSecretSharing require " \
                                     "shared_party_num > 1"
        self.shared_party_num = shared_party_num
        self.maximum = 2**size
        self.mod_number = 2 * self.maximum + 1
        self.epsilon = 1e8
        self.mod_funs = np.vectorize(lambda x: x % self.mod_number)
        self.float2fixedpoint = np.vectorize(self._float2fixedpoint)
        self.fixedpoint2float = np.vectorize(self._fixedpoint2float)

    def secret_split(self, secret):
        """n-1 uniform int64 frames plus the frame that completes the sum
        (secret_sharing.py:38-71)."""
        if isinstance(secret, dict):
            frames = [dict() for _ in range(self.shared_party_num)]
            for key, value in secret.items():
                for idx, part in enumerate(self.secret_split(value)):
                    frames[idx][key] = part
            return frames
        if torch is not None and isinstance(secret, torch.Tensor):
            secret = secret.numpy()
        if isinstance(secret, (list, np.ndarray)):
            secret = np.asarray(secret)
            shape = [self.shared_party_num - 1] + list(secret.shape)
        else:
            shape = [self.shared_party_num - 1]
        fixed = self.float2fixedpoint(secret)
        frames = np.random.randint(low=0, high=self.mod_number, size=shape)
        last = self.mod_funs(fixed - self.mod_funs(np.sum(frames, axis=0)))
        return np.append(frames, np.expand_dims(last, axis=0), axis=0)

    def secret_reconstruct(self, secret_seq):
        """Sum the frames key by key and map back (secret_sharing.py:73-86)."""
        assert len(secret_seq) == self.shared_party_num
        merged = secret_seq[0].copy()
        if isinstance(merged, dict):
            for key in merged:
                acc = secret_seq[0][key]
                for idx in range(1, len(secret_seq)):
                    acc += secret_seq[idx][key]
                merged[key] = self.fixedpoint2float(acc)
        return merged

    def _float2fixedpoint(self, x):
        x = round(x * self.epsilon, 0)
        assert abs(x) < self.maximum
        return x % self.mod_number

    def _fixedpoint2float(self, x):
        x = x % self.mod_number
        if x > self.maximum:
            return -1 * (self.mod_number - x) / self.epsilon
        return x / self.epsilon


def ss_params(recover_fun):
    """(mod, maximum, epsilon) as doubles for the device recovery, from
    ``AdditiveSecretSharing(...).fixedpoint2float`` — this package's or the
    reference's (both are np.vectorize of the bound _fixedpoint2float).
    Other recover functions have no device path and raise."""
    fn = getattr(recover_fun, 'pyfunc', None)
    owner = getattr(fn, '__self__', None)
    if owner is not None and getattr(fn, '__name__', '') == \
            '_fixedpoint2float' and hasattr(owner, 'mod_number') and \
            hasattr(owner, 'maximum') and hasattr(owner, 'epsilon'):
        # numpy converts the Python ints to float64 in `x % mod_number` and
        # `mod_number - x` (2·2^60 + 1 rounds to 2^61)
        return (float(owner.mod_number), float(owner.maximum),
                float(owner.epsilon))
    raise NotImplementedError(
        'device secret-sharing recovery supports '
        'AdditiveSecretSharing.fixedpoint2float only (got %r)' % recover_fun)
