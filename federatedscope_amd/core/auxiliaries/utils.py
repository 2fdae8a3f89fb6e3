"""Helpers the aggregation path shares with the reference.

Mirrors federatedscope/core/auxiliaries/utils.py:95-111 (param2tensor,
merge_param_dict).  The gRPC wire format ships tensors as base64-encoded
pickles (federatedscope/core/message.py:8-9,118-120); they are decoded here
with a restricted unpickler that only admits torch's tensor-rebuild helpers,
so a crafted message cannot execute code.
"""
import base64
import collections
import io
import pickle

import torch


def _storage_from_bytes(b):
    return torch.load(io.BytesIO(b), weights_only=True)


class _TensorUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ('torch._utils', '_rebuild_tensor_v2'): torch._utils._rebuild_tensor_v2,
        ('torch.storage', '_load_from_bytes'): _storage_from_bytes,
        ('collections', 'OrderedDict'): collections.OrderedDict,
    }

    def find_class(self, module, name):
        fn = self._ALLOWED.get((module, name))
        if fn is None:
            raise pickle.UnpicklingError(
                'refusing to unpickle %s.%s in a model update' % (module, name))
        return fn


def b64_to_tensor(s):
    """Decode one b64serializer payload (message.py:8-9) on the host: the
    framing walker of core/compression/b64wire reads the pickle framing and
    only the storage bytes are base64-decoded (no pickle machinery runs).
    A payload it does not recognise (e.g. another pickle protocol's bytes
    encoding) goes through the restricted unpickler; if that fails too, the
    framing error is raised."""
    from ..compression.b64wire import FramingError, decode_b64
    try:
        return decode_b64(s)
    except FramingError as e:
        try:
            return _TensorUnpickler(io.BytesIO(base64.b64decode(s))).load()
        except Exception:
            raise e from None


def param_meta(param):
    """What param2tensor would return, as far as shape, dtype and device
    go — without decoding base64 text (a meta tensor for it)."""
    if isinstance(param, str):
        from ..compression.b64wire import FramingError, parse_b64
        try:
            return parse_b64(param).meta()
        except FramingError:
            pass
    return param2tensor(param)


def param2tensor(param):
    """list → FloatTensor, int → long, float → float, str → decoded tensor;
    tensors pass through (utils.py:95-105)."""
    if isinstance(param, list):
        param = torch.FloatTensor(param)
    elif isinstance(param, int):
        param = torch.tensor(param, dtype=torch.long)
    elif isinstance(param, float):
        param = torch.tensor(param, dtype=torch.float)
    elif isinstance(param, str):
        param = b64_to_tensor(param)
    return param


def as_float_tensor(param):
    """The robust and async rules' cast of a client value to fp32
    (``x.float()`` for tensors, ``torch.FloatTensor(x)`` otherwise:
    asyn_clients_avg_aggregator.py:74-77, krum_aggregator.py:48-53)."""
    t = param2tensor(param)
    if isinstance(t, torch.Tensor):
        return t.float()
    import numpy as np
    return torch.as_tensor(np.asarray(t)).float()


def as_float_upload(param):
    """as_float_tensor for staging: base64 text whose framing is already
    fp32 stays text (the device decodes it, core/compression/b64wire)."""
    if isinstance(param, str) and param_meta(param).dtype == torch.float32:
        return param
    return as_float_tensor(param)


def merge_param_dict(raw_param, filtered_param):
    """Overlay the aggregate onto the model state_dict (utils.py:108-111)."""
    for key in filtered_param.keys():
        raw_param[key] = filtered_param[key]
    return raw_param
