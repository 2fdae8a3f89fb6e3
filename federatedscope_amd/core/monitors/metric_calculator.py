"""Update-dissimilarity metrics of a round, on the GPU (drop-ins for
calc_blocal_dissim / calc_l2_dissim,
federatedscope/core/monitors/metric_calculator.py:309-372).

Both read every client's update once more after (or instead of) the
aggregation.  Device-resident client tensors (GPU dicts, or the server's
staged stack rows) are read in place through a per-key pointer table
(ops.KeyTable, no copy); host dicts are staged into a device stack first.
The per-client, per-key
‖local − last‖² come from one fsagg_delta_sqnorm_f32 pass (fp64 sums), the
global update Σ_i w_i (local_i − last) from fsagg_delta_wsum_f32 (the
reference's fp32 op order, bit-exact) and its per-key ‖·‖² from a second
fsagg_delta_sqnorm_f32 over that one row.  The reference sums squares in
fp32 with ATen's reduction order, so the results are tolerance-pinned
(≤ 1e-5 relative; tests/test_gpu_wire.py).
"""
from collections import OrderedDict

import numpy as np
import torch

from ... import ops
from ...layout import BucketLayout, ClientStack
from ..auxiliaries.utils import param2tensor

_STACKS = {}


def _staged(last_model, local_updated_models):
    from ..aggregators._engine import compute_device
    dev = compute_device()
    keys = list(local_updated_models[0][1].keys())
    template = OrderedDict((k, param2tensor(last_model[k]).float())
                           for k in keys)
    lay = BucketLayout(template)
    n = len(local_updated_models)
    sig = (lay.signature(), str(dev))
    st = _STACKS.get(sig)
    if st is None or st.capacity < n:
        st = ClientStack(lay, n, dev)
        st.slab.zero_()
        _STACKS.clear()
        _STACKS[sig] = st
    st.load_many([OrderedDict((k, param2tensor(m[k]).float()) for k in keys)
                  for _, m in local_updated_models])
    last = torch.zeros(lay.numel, dtype=torch.float32, device=dev)
    lay.pack_device(template, last)
    return lay, st, last, keys


def _in_place(last_model, local_updated_models):
    """A KeyTable over the clients' own tensors when every one of them is a
    contiguous fp32 tensor on the compute device (device-resident dicts,
    StagedUpdate views of the server's stack) — no staging copy; else
    None (the caller stages)."""
    from ..aggregators._engine import compute_device
    dev = compute_device()
    if dev.type != 'cuda':
        return None
    keys = list(local_updated_models[0][1].keys())
    try:
        table = ops.KeyTable([[m[k] for k in keys]
                              for _, m in local_updated_models], dev)
    except (KeyError, TypeError, AttributeError, ValueError):
        return None
    base = [param2tensor(last_model[k]).float().to(table.device).contiguous()
            for k in keys]
    if any(b.numel() != sz for b, sz in zip(base, table.sizes)):
        return None
    return table, base, keys


def calc_l2_dissim(last_model, local_updated_models):
    """‖cat_k(local_k − last_k)‖₂ per client, and their mean
    (metric_calculator.py:360-372)."""
    n = len(local_updated_models)
    kt = _in_place(last_model, local_updated_models)
    if kt is not None:
        sq = ops.delta_sqnorm_keys(kt[0], base=kt[1])
    else:
        lay, st, last, keys = _staged(last_model, local_updated_models)
        sq = ops.delta_sqnorm(st.rows(list(range(n))), lay.segments(),
                              base=last)
    raw = [float(np.sqrt(v)) for v in sq.sum(1).cpu().tolist()]
    return {'raw': raw, 'mean': np.mean(raw)}


def calc_blocal_dissim(last_model, local_updated_models):
    """B-local dissimilarity per key [Li et al., FedProx]
    (metric_calculator.py:309-357):
    sqrt(Σ_i w_i ‖g_ik‖² / ‖Σ_i w_i g_ik‖²), g_i = local_i − last,
    w = sample sizes normalised in float64."""
    n = len(local_updated_models)
    weights = np.asarray([tp[0] for tp in local_updated_models])
    weights = weights / np.sum(weights)
    kt = _in_place(last_model, local_updated_models)
    # the norms and the global update in one read of the clients
    if kt is not None:
        table, base, keys = kt
        segs = table.offsets
        g = torch.empty(table.numel, dtype=torch.float32, device=table.device)
        sq = ops.delta_sqnorm_wsum_keys(table, [float(w) for w in weights],
                                        base, g).cpu().numpy()
    else:
        lay, st, last, keys = _staged(last_model, local_updated_models)
        rows = st.rows(list(range(n)))
        segs = lay.segments()
        g = torch.empty(lay.numel, dtype=torch.float32, device=last.device)
        sq = ops.delta_sqnorm_wsum(rows, [float(w) for w in weights], segs,
                                   last, g).cpu().numpy()
    gsq = ops.delta_sqnorm(ops.RowTable.from_tensors([g]), segs)
    gsq = gsq.cpu().numpy()[0]
    out = dict()
    for s, k in enumerate(keys):
        avg = 0.0
        for i in range(n):
            avg += weights[i] * sq[i][s]
        out[k] = np.sqrt(avg / gsq[s])
    return out
