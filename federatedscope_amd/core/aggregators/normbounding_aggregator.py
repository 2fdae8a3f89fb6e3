"""Norm bounding (federatedscope/core/aggregators/
normbounding_aggregator.py:10-70) on the GPU.

Per client, the L2 norm of the flattened update over the server model's keys
(fp64 two-level reduction, rounded to fp32 like torch.norm's result); if it
exceeds the bound the client is scaled by fl32(bound / norm).  The scale is
applied inside the weighted-sum kernel as a per-client prescale
(fl32(fl32(x·s)·w)), then init + avg is fused into the epilogue."""
import math

from ._engine import _first_device
from .clients_avg_aggregator import ClientsAvgAggregator
from ... import ops

import numpy as np


class NormboundingAggregator(ClientsAvgAggregator):
    def __init__(self, model=None, device='cpu', config=None):
        super().__init__(model, device, config)
        self.norm_bound = config.aggregator.BFT_args.normbounding_norm_bound

    def aggregate(self, agg_info):
        models = agg_info["client_feedback"]
        out_dev = _first_device(models[0][1])
        init = self.model.state_dict()
        st = self._stage_all(models)
        layout = st.layout
        if [k for k in init if k in models[0][1]] != layout.keys:
            raise NotImplementedError(
                'norm bounding with client keys that differ from the server '
                'model keys')
        n = len(models)
        sq = self._sqnorms(st).sum(1).cpu().numpy()
        pre = []
        bound32 = np.float32(self.norm_bound)
        for i in range(n):
            norm = np.float32(math.sqrt(float(sq[i])))
            if norm > self.norm_bound:
                pre.append(float(np.float32(bound32 / norm)))
            else:
                pre.append(1.0)
        weights = self._weights(models)
        layout, flat, extra, keys = self._weighted_avg_device(
            models, weights, as_float=True, base_model=init, prescale=pre,
            staged=st)
        return self._emit(layout, flat, keys, out_dev, extra)
