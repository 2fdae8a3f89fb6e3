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
            return self._ss_avg(models, recover_fun)
        weights = self._weights(models)
        out_dev = _first_device(models[0][1])
        layout, flat, extra, keys = self._weighted_avg_device(models, weights)
        return self._emit(layout, flat, keys, out_dev, extra)

    def _ss_avg(self, models, recover_fun):
        """The use_ss branch (clients_avg_aggregator.py:79-98): every upload
        is the client's share sum of sample_size·params in fixed point;
        weight 1.0 — or 1/n when ignore_weight is set too, which the
        reference tests first (:77-82) — Σ in float64 (numpy), then
        fixedpoint2float, ÷ total, fp32 — fused in fsagg_ss_recover_f32.
        Without a recover function the float64 sums are returned (the
        reference leaves them numpy)."""
        from ..secret_sharing import ss_params
        dev = self.compute_device
        total = 0
        for size, _ in models:
            total += size
        w = 1.0 / len(models) if self.cfg.federate.ignore_weight else 1.0
        params = ss_params(recover_fun) if recover_fun else None
        avg = OrderedDict()
        keys = list(models[0][1].keys())
        out_dev = torch.device('cpu')
        for key in keys:
            shares = [_share_to_device(m[key], dev) for _, m in models
                      if key in m]
            if params is None:
                avg[key] = ops.ss_recover(shares, 1.0, 0.0, 1.0, 1.0,
                                          recover=False,
                                          weight=w).to(out_dev)
            else:
                mod, maximum, eps = params
                avg[key] = ops.ss_recover(shares, mod, maximum, eps,
                                          float(total),
                                          weight=w).to(out_dev)
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


_DT_CODE = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2,
            torch.float64: 3, torch.int64: 4}


class OnlineClientsAvgAggregator(ClientsAvgAggregator):
    """Streaming running mean (clients_avg_aggregator.py:103-148):
    m = (cnt*m + s*x) / (cnt + s) per client, on the GPU.  fp32 keys with
    fp32 uploads live in one bucket and take one launch per upload; any
    other dtype pair follows ATen's promotion per key
    (fsagg_online_inc_typed) — an int64 counter becomes a float32 mean, an
    fp64 upload promotes its key."""
    def __init__(self, model=None, device='cpu', src_device='cpu',
                 config=None):
        super().__init__(model, device, config)
        self.src_device = src_device

    def reset(self):
        sd = self.model.state_dict()
        self._layout_m = self._layout(sd)
        dev = self.compute_device
        self._m = torch.zeros(self._layout_m.numel, dtype=torch.float32,
                              device=dev)
        # keys held outside the fp32 bucket (other dtypes, or promoted)
        self._m_other = OrderedDict(
            (k, torch.zeros(param2tensor(sd[k]).shape, dtype=dt, device=dev))
            for k, dt in self._layout_m.other.items())
        self._keys = list(sd.keys())
        self._x = torch.zeros_like(self._m)
        self.cnt = 0

    def _typed_inc(self, k, m, x, sample_size):
        """One key through fsagg_online_inc_typed; returns the new value."""
        from ... import _lib as L
        if m.dtype not in _DT_CODE or x.dtype not in _DT_CODE:
            raise TypeError('online aggregation of %s/%s key %r' %
                            (m.dtype, x.dtype, k))
        ct = torch.promote_types(m.dtype, x.dtype)
        odt = torch.float32 if ct == torch.int64 else ct
        x = x.to(m.device).contiguous()
        m = m.contiguous()
        out = m if odt == m.dtype else torch.empty(m.shape, dtype=odt,
                                                   device=m.device)
        if m.numel() != x.numel():
            raise ValueError('upload of key %r has %d elements, the model '
                             '%d' % (k, x.numel(), m.numel()))
        L.check(L.load().fsagg_online_inc_typed(
            m.data_ptr(), _DT_CODE[m.dtype], x.data_ptr(), _DT_CODE[x.dtype],
            out.data_ptr(), _DT_CODE[ct], int(self.cnt), int(sample_size),
            m.numel(), ops._stream(m.device)), 'fsagg_online_inc_typed')
        return out

    def inc(self, content):
        if not isinstance(content, tuple):
            raise TypeError(
                "{} is not a tuple (sample_size, model_para)".format(content))
        sample_size, model_params = content
        lay = self._layout_m
        fast = []
        for k in lay.keys:
            if k in model_params and k not in self._m_other and \
                    param2tensor(model_params[k]).dtype == torch.float32:
                fast.append(k)
        dev = self._m.device
        ups = {k: param2tensor(model_params[k]) for k in fast}
        if fast and all(t.device == dev and t.is_contiguous() and
                        t.data_ptr() % 16 == 0 for t in ups.values()):
            # uploads already on the device: each key's running mean reads
            # the upload in place (12 B per parameter, no packing copy)
            for k in fast:
                o, m = lay.offsets[k], lay.numels[k]
                if m:            # an empty key's tensor may have no storage
                    ops.online_inc(self._m[o:o + m], ups[k].reshape(-1),
                                   self.cnt, sample_size)
        elif fast:
            lay.pack_device(OrderedDict((k, ups[k]) for k in fast), self._x)
            if len(fast) == len(lay.keys):
                ops.online_inc(self._m, self._x, self.cnt, sample_size)
            else:
                for k in fast:
                    o, m = lay.offsets[k], lay.numels[k]
                    ops.online_inc(self._m[o:o + m], self._x[o:o + m],
                                   self.cnt, sample_size)
        for k in self._keys:
            if k not in model_params or k in fast:
                continue
            x = param2tensor(model_params[k])
            if k in self._m_other:
                m = self._m_other[k]
            else:                    # an fp32 bucket key, non-fp32 upload
                o, n = lay.offsets[k], lay.numels[k]
                m = self._m[o:o + n].view(lay.shapes[k])
            new = self._typed_inc(k, m, x, sample_size)
            if k in self._m_other or new.dtype != torch.float32:
                self._m_other[k] = new          # promoted keys leave the
            elif new is not m:                  # bucket for good
                m.copy_(new)
        self.cnt += sample_size

    @property
    def maintained(self):
        return self._emit(self._layout_m, self._m, self._keys,
                          torch.device(self.src_device), self._m_other)

    def aggregate(self, agg_info):
        return self.maintained
