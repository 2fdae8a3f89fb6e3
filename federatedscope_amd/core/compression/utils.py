"""Symmetric uniform quantisation of uploads (drop-in for
federatedscope/core/compression/utils.py).

* ``symmetric_uniform_quantization`` is the CLIENT side (utils.py:8-61): it
  stays a restatement in torch ops on whatever device the model lives —
  clients are not the server's hot path.
* ``symmetric_uniform_dequantization`` is the SERVER side (utils.py:64-90,
  called from Server.callback_funcs_model_para, server.py:946-960): the
  ``value * alpha`` of every ``*.weight_quant`` key runs in libfsagg's
  fsagg_wire_unpack_f32 (fl32(float(q) * scale), bit-identical to the
  reference's int8/int16 × fp32 0-dim tensor product).  Host tensors in give
  host tensors out.  The server's staged path (WireStager) decodes uploads
  straight into the device client stack instead.
"""
import logging

import torch

from ... import _lib as L
from ... import ops

logger = logging.getLogger(__name__)


def _symmetric_uniform_quantization(x, nbits, stochastic=False):
    """utils.py:8-29, op for op."""
    assert (torch.isnan(x).sum() == 0)
    assert (torch.isinf(x).sum() == 0)
    c = torch.max(torch.abs(x))
    s = c / (2**(nbits - 1) - 1)
    if s == 0:
        return x, s
    qx = x / s
    if stochastic:
        noise = qx.new(qx.shape).uniform_(-0.5, 0.5)
        qx.add_(noise)
    qx.clamp_(-(2**(nbits - 1) - 1), (2**(nbits - 1) - 1)).round_()
    return qx, s


def symmetric_uniform_quantization(state_dict, nbits=8):
    """utils.py:32-61: quantise the weights of conv / fc layers to int8 or
    int16 with one fp32 scale per tensor."""
    if nbits == 8:
        quant_data_type = torch.int8
    elif nbits == 16:
        quant_data_type = torch.int16
    else:
        logger.info(f'The provided value of nbits ({nbits}) is invalid, and '
                    f'we change it to 8')
        nbits = 8
        quant_data_type = torch.int8
    quant_state_dict = dict()
    for key, value in state_dict.items():
        if ('fc' in key or 'conv' in key) and 'weight' == key.split('.')[-1]:
            q_weight, w_s = _symmetric_uniform_quantization(value, nbits=nbits)
            quant_state_dict[key.replace(
                'weight', 'weight_quant')] = q_weight.type(quant_data_type)
            quant_state_dict[key.replace('weight', 'weight_scale')] = w_s
        else:
            quant_state_dict[key] = value
    return quant_state_dict


def scale_to_f32(alpha):
    """The fp32 value the reference multiplies by: the 0-dim scale tensor
    itself, or a Python number rounded to fp32 (ATen casts a scalar operand
    to the float result type)."""
    if isinstance(alpha, torch.Tensor):
        return float(alpha.detach().to('cpu', torch.float32).reshape(()))
    return float(torch.tensor(float(alpha), dtype=torch.float32))


def dequantize_tensor(value, alpha, device=None):
    """fl32(float(q) * alpha) for one int8/int16 tensor on the GPU; the
    result is returned on the device ``value`` came from."""
    from ..aggregators._engine import compute_device
    if value.dtype not in (torch.int8, torch.int16):
        raise TypeError('weight_quant must be int8 or int16 (got %s)' %
                        value.dtype)
    dev = compute_device(device if device is not None else (
        value.device if value.device.type == 'cuda' else None))
    q = value.detach().contiguous().to(dev)
    kind = L.FSAGG_WIRE_I8 if q.dtype == torch.int8 else L.FSAGG_WIRE_I16
    out = torch.empty(q.shape, dtype=torch.float32, device=dev)
    n = q.numel()
    if n:
        segs = ops.wire_segments([(0, 0, n, kind, 0)], dev)
        scales = torch.tensor([scale_to_f32(alpha)], dtype=torch.float32,
                              device=dev)
        src = q.view(-1).view(torch.uint8)
        ops.wire_unpack(src, segs, 1, n, scales, out.view(-1),
                        src_bytes=src.numel(), max_dst=n)
    return out if value.device.type == 'cuda' else out.to(value.device)


def symmetric_uniform_dequantization(state_dict):
    """utils.py:64-90: ``x.weight_quant * x.weight_scale`` → ``x.weight``
    (same key order), on the GPU."""
    dequantizated_state_dict = dict()
    for key, value in state_dict.items():
        if 'weight_quant' in key:
            alpha = state_dict[key.replace('weight_quant', 'weight_scale')]
            dequantizated_state_dict[key.replace(
                'weight_quant', 'weight')] = dequantize_tensor(value, alpha)
        elif 'weight_scale' in key:
            pass
        else:
            dequantizated_state_dict[key] = value
    return dequantizated_state_dict
