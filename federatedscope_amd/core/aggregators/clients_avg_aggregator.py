"""FedAvg drop-ins: ClientsAvgAggregator and OnlineClientsAvgAggregator.

Reference: federatedscope/core/aggregators/clients_avg_aggregator.py.
The reduction runs in libfsagg's fsagg_weighted_sum_f32 (bit-identical to the
reference's ATen CPU loop: per element, client-list order, every multiply and
add rounded to fp32, no FMA).
"""
from collections import OrderedDict

import torch

from ... import ops
from ..auxiliaries.utils import param2tensor
from ._engine import DeviceEngine, _first_device, fedavg_weights
from .aggregator import Aggregator, _ModelIO


class ClientsAvgAggregator(DeviceEngine, _ModelIO, Aggregator):
    """Vanilla FedAvg [McMahan et al., 2017] on the GPU
    (clients_avg_aggregator.py:7-100)."""
    def __init__(self, model=None, device='cpu', config=None):
        Aggregator.__init__(self)
        self.model = model
        self.device = device
        self.cfg = config
        self._engine_init(device)

    def aggregate(self, agg_info):
        models = agg_info["client_feedback"]
        recover_fun = agg_info['recover_fun'] if (
            'recover_fun' in agg_info and self.cfg.federate.use_ss) else None
        return self._para_weighted_avg(models, recover_fun=recover_fun)

    def _weights(self, models):
        fed = self.cfg.federate
        return fedavg_weights([s for s, _ in models],
                              ignore_weight=fed.ignore_weight)

    def _para_weighted_avg(self, models, recover_fun=None):
        """Weighted average of the client dicts (clients_avg_aggregator.py:60-100).

        Returns a state_dict in client 0's key order on client 0's device."""
        if self.cfg.federate.use_ss:
            if self.cfg.federate.ignore_weight:
                raise NotImplementedError(
                    'use_ss with ignore_weight (1/n-weighted fixed-point '
                    'shares) has no device path')
            return self._ss_avg(models, recover_fun)
        weights = self._weights(models)
        out_dev = _first_device(models[0][1])
        layout, flat, extra, keys = self._weighted_avg_device(models, weights)
        return self._emit(layout, flat, keys, out_dev, extra)

    def _ss_avg(self, models, recover_fun):
        """The use_ss branch (clients_avg_aggregator.py:79-98): every upload
        is the client's share sum of sample_size·params in fixed point;
        weight 1.0, Σ in float64 (numpy), then fixedpoint2float, ÷ total,
        fp32 — fused in fsagg_ss_recover_f32.  Without a recover function
        the float64 sums are returned (the reference leaves them numpy)."""
        from ..secret_sharing import ss_params
        dev = self.compute_device
        total = 0
        for size, _ in models:
            total += size
        params = ss_params(recover_fun) if recover_fun else None
        avg = OrderedDict()
        keys = list(models[0][1].keys())
        out_dev = torch.device('cpu')
        for key in keys:
            shares = [_share_to_device(m[key], dev) for _, m in models
                      if key in m]
            if params is None:
                avg[key] = ops.ss_recover(shares, 1.0, 0.0, 1.0, 1.0,
                                          recover=False).to(out_dev)
            else:
                mod, maximum, eps = params
                avg[key] = ops.ss_recover(shares, mod, maximum, eps,
                                          float(total)).to(out_dev)
        return avg


def _share_to_device(x, dev):
    """A client's share sum (numpy int64/float64 array, or a tensor of those
    dtypes) as a contiguous device tensor."""
    import numpy as np
    if isinstance(x, torch.Tensor):
        t = x.detach()
    else:
        a = np.asarray(x)
        if a.dtype not in (np.int64, np.float64):
            raise NotImplementedError('secret-sharing share of dtype %s' %
                                      a.dtype)
        t = torch.from_numpy(np.ascontiguousarray(a))
    if t.dtype not in (torch.int64, torch.float64):
        raise NotImplementedError('secret-sharing share of dtype %s' %
                                  t.dtype)
    return t.to(dev).contiguous()


class OnlineClientsAvgAggregator(ClientsAvgAggregator):
    """Streaming running mean (clients_avg_aggregator.py:103-148):
    m = (cnt*m + s*x) / (cnt + s) per client, on the GPU."""
    def __init__(self, model=None, device='cpu', src_device='cpu',
                 config=None):
        super().__init__(model, device, config)
        self.src_device = src_device

    def reset(self):
        sd = self.model.state_dict()
        self._layout_m = self._layout(sd)
        self._m = torch.zeros(self._layout_m.numel, dtype=torch.float32,
                              device=self.compute_device)
        # non-fp32 model entries (e.g. BN counters) stay zeros of their dtype
        self._m_other = OrderedDict(
            (k, torch.zeros_like(sd[k], device=self.src_device))
            for k in self._layout_m.other)
        self._keys = list(sd.keys())
        self._x = torch.zeros_like(self._m)
        self.cnt = 0

    def inc(self, content):
        if not isinstance(content, tuple):
            raise TypeError(
                "{} is not a tuple (sample_size, model_para)".format(content))
        sample_size, model_params = content
        lay = self._layout_m
        for k in lay.other:
            if k in model_params:
                raise NotImplementedError(
                    'online aggregation of non-fp32 key %r' % k)
        lay.pack_device(OrderedDict(
            (k, param2tensor(model_params[k])) for k in lay.keys
            if k in model_params), self._x)
        if all(k in model_params for k in lay.keys):
            ops.online_inc(self._m, self._x, self.cnt, sample_size)
        else:
            for k in lay.keys:
                if k not in model_params:
                    continue
                o, m = lay.offsets[k], lay.numels[k]
                ops.online_inc(self._m[o:o + m], self._x[o:o + m], self.cnt,
                               sample_size)
        self.cnt += sample_size

    @property
    def maintained(self):
        return self._emit(self._layout_m, self._m, self._keys,
                          torch.device(self.src_device), self._m_other)

    def aggregate(self, agg_info):
        return self.maintained
