"""Server side of the symmetric uniform quantisation of uploads (drop-in
for the dequantisation half of federatedscope/core/compression/utils.py).

* Quantisation is the CLIENTS' job (utils.py:8-61) and is not rebuilt here:
  FederatedScope's own client code keeps producing the wire dicts.
* ``symmetric_uniform_dequantization`` is the SERVER side (utils.py:64-90,
  called from Server.callback_funcs_model_para, server.py:946-960): the
  ``value * alpha`` of every ``*.weight_quant`` key runs in libfsagg's
  fsagg_wire_unpack_f32 (fl32(float(q) * scale), bit-identical to the
  reference's int8/int16 × fp32 0-dim tensor product).  Host tensors in give
  host tensors out.  The server's staged path (WireStager) decodes uploads
  straight into the device client stack instead.
"""
import torch

from ... import _lib as L
from ... import ops


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
