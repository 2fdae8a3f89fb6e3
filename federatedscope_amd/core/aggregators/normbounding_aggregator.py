"""Norm bounding (federatedscope/core/aggregators/
normbounding_aggregator.py:10-70) on the GPU.

Per client, the L2 norm of the flattened update over the server model's keys
the client holds (per-(client, key) fp64 sums, rounded to fp32 like
torch.norm's result); if it exceeds the bound the client is scaled by
fl32(bound / norm).  When every client holds exactly the server's keys the
scale is applied inside the weighted-sum kernel as a per-client prescale
(fl32(fl32(x·s)·w)) and init + avg is fused into its epilogue.  Otherwise
the reference's reconstruction is followed literally (:49-70): a scaled
client becomes a copy of the SERVER model with its own keys replaced by the
scaled values (keys it lacks come back as the server's), an unscaled client
stays as uploaded, and the weighted average runs over those dicts."""
import math
from collections import OrderedDict

import numpy as np
import torch

from ... import ops
from ..auxiliaries.utils import as_float_tensor, param2tensor
from ._engine import _first_device
from .clients_avg_aggregator import ClientsAvgAggregator


class NormboundingAggregator(ClientsAvgAggregator):
    def __init__(self, model=None, device='cpu', config=None):
        super().__init__(model, device, config)
        self.norm_bound = config.aggregator.BFT_args.normbounding_norm_bound

    def _rates(self, sq):
        """The reference's ``self.norm_bound / torch.norm(param)`` per client
        whose norm exceeds the bound (else None), with norm =
        fl32(sqrt(Σ squares)) as torch.norm returns it.  A Python float over
        a 0-dim tensor is Tensor.__rtruediv__ = reciprocal() * other:
        fl32(fl32(1 / norm) · fl32(bound)), which differs from
        fl32(bound / norm) in the last bit for ~16 % of norms."""
        bound32 = np.float32(self.norm_bound)
        one = np.float32(1.0)
        out = []
        for v in sq:
            norm = np.float32(math.sqrt(float(v)))
            out.append(float(np.float32(np.float32(one / norm) * bound32))
                       if norm > self.norm_bound else None)
        return out

    def aggregate(self, agg_info):
        models = agg_info["client_feedback"]
        out_dev = _first_device(models[0][1])
        init = self.model.state_dict()
        ikeys = list(init.keys())
        if all(list(m.keys()) == ikeys for _, m in models):
            return self._aggregate_same_keys(models, init, out_dev)
        return self._aggregate_general(models, init, out_dev)

    def _aggregate_same_keys(self, models, init, out_dev):
        st = self._stage_all(models)
        # the rates stay on the device: no host round trip between the norm
        # pass and the weighted sum
        pre = ops.normbound_prescale(self._sqnorms(st), self.norm_bound)
        weights = self._weights(models)
        layout, flat, extra, keys = self._weighted_avg_device(
            models, weights, as_float=True, base_model=init, prescale=pre,
            staged=st)
        return self._emit(layout, flat, keys, out_dev, extra)

    def _aggregate_general(self, models, init, out_dev):
        # norms over the server keys each client holds
        dicts = [m for _, m in models]
        flat_init = OrderedDict((k, as_float_tensor(param2tensor(v)))
                                for k, v in init.items())
        lay = self._layout(flat_init, as_float=True)
        cl = [OrderedDict((k, d[k]) for k in init if k in d) for d in dicts]
        present = [[k in d for k in lay.keys] for d in cl]
        stack = self._stack(lay, cl, as_float=True)
        rs = ops.RowSet.from_stack(stack, range(len(cl)), present=present)
        sq = ops.rows_sqnorm(rs).sum(1).cpu().numpy()
        rates = self._rates(sq)
        dev = self.compute_device
        tmp = []
        for i, (size, d) in enumerate(models):
            if rates[i] is None:
                tmp.append((size, d))
                continue
            # fl32(rate · x) of the client's keys, in its stack row
            row = torch.empty(lay.numel, dtype=torch.float32, device=dev)
            ops.weighted_sum_rows(rs.subset([i]), [rates[i]], row)
            views = lay.unpack(row)
            rec = OrderedDict()
            for k in init:            # a deepcopy of the server model ...
                rec[k] = views[k] if k in cl[i] else \
                    param2tensor(init[k]).to(dev)   # ... with its keys set
            tmp.append((size, rec))
        weights = self._weights(tmp)
        layout, flat, extra, keys = self._weighted_avg_device(
            tmp, weights, as_float=True, base_model=init)
        return self._emit(layout, flat, keys, out_dev, extra)
