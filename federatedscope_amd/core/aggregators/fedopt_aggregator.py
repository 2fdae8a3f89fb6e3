"""FedOpt [Reddi et al., 2021] (federatedscope/core/aggregators/
fedopt_aggregator.py:7-44) with the server-optimizer step on the GPU.

aggregate(): FedAvg of the clients into a device bucket (bit-exact, as
ClientsAvgAggregator), then ONE fused pass fsagg_server_opt_step_f32 that
forms g = model − avg and applies torch.optim's SGD (momentum, dampening,
nesterov, weight decay) or Adam update to the server model's parameter
bucket and the optimizer-state buckets, which stay resident in HBM across
rounds.  The updated parameters are written back into ``self.model`` and
``self.model.state_dict()`` is returned, as the reference does.

Optimizer config: ``config.fedopt.optimizer`` = {type, lr, **kwargs} as in
get_optimizer (core/auxiliaries/optimizer_builder.py:19-60); annealing:
StepLR(step_size, gamma) stepped once per aggregation (:14-22, :43-44).
"""
import ctypes
from collections import OrderedDict

import torch

from ... import _lib as L
from ...ops import _check_f32_cuda, _stream
from ._engine import fedavg_weights
from .clients_avg_aggregator import ClientsAvgAggregator

_SUPPORTED = ('SGD', 'Adam')


def _opt_cfg(optimizer_cfg):
    if isinstance(optimizer_cfg, dict):
        d = dict(optimizer_cfg)
    else:
        d = {k: v for k, v in vars(optimizer_cfg).items()
             if not k.startswith('__')}
    for k in ('__help_info__', '__cfg_check_funcs__', 'is_ready_for_run'):
        d.pop(k, None)
    return d


class FedOptAggregator(ClientsAvgAggregator):
    def __init__(self, config, model, device='cpu'):
        super().__init__(model, device, config)
        opt = _opt_cfg(config.fedopt.optimizer)
        self.opt_type = opt.pop('type')
        self.lr0 = float(opt.pop('lr'))
        if self.opt_type not in _SUPPORTED:
            raise NotImplementedError(
                'FedOpt server optimizer %r is not on the device path '
                '(supported: %s)' % (self.opt_type, ', '.join(_SUPPORTED)))
        self.kw = opt
        if self.opt_type == 'SGD':
            self.momentum = float(opt.get('momentum', 0.0))
            self.dampening = float(opt.get('dampening', 0.0))
            self.weight_decay = float(opt.get('weight_decay', 0.0))
            self.nesterov = bool(opt.get('nesterov', False))
            if opt.get('maximize', False):
                raise NotImplementedError('maximize=True')
        else:
            betas = opt.get('betas', (0.9, 0.999))
            self.beta1, self.beta2 = float(betas[0]), float(betas[1])
            self.eps = float(opt.get('eps', 1e-8))
            self.weight_decay = float(opt.get('weight_decay', 0.0))
            if opt.get('amsgrad', False) or opt.get('maximize', False):
                raise NotImplementedError('amsgrad / maximize')
        fo = config.fedopt
        self._annealing = bool(getattr(fo, 'annealing', False))
        self._anneal_step = int(getattr(fo, 'annealing_step_size', 2000))
        self._anneal_gamma = float(getattr(fo, 'annealing_gamma', 0.5))
        self._rounds = 0
        self._state = {}     # layout signature -> (s0, s1, steps)

    def _lr(self):
        if not self._annealing:
            return self.lr0
        return self.lr0 * self._anneal_gamma ** (self._rounds //
                                                 self._anneal_step)

    def aggregate(self, agg_info):
        models = agg_info["client_feedback"]
        weights = fedavg_weights([s for s, _ in models],
                                 self.cfg.federate.ignore_weight)
        layout, avg, extra, keys = self._weighted_avg_device(models, weights)
        named = OrderedDict(self.model.named_parameters())
        step_keys = [k for k in named if k in layout.keys]
        for k in named:
            if k in extra:
                raise NotImplementedError('FedOpt on non-fp32 parameter %r' %
                                          k)
        param = self._bucket(layout, OrderedDict(
            (k, named[k].detach() if k in named else torch.zeros(
                layout.shapes[k])) for k in layout.keys))
        sig = layout.signature()
        if sig not in self._state:
            s0 = torch.zeros_like(param)
            s1 = torch.zeros_like(param) if self.opt_type == 'Adam' else None
            self._state[sig] = [s0, s1, 0]
        st = self._state[sig]
        hp = self._params(first=(st[2] == 0), step=st[2] + 1)
        lib = L.load()
        for k in step_keys:      # per key: params the optimizer owns
            o, m = layout.offsets[k], layout.numels[k]
            for t in (param, avg, st[0]):
                _check_f32_cuda(t[o:o + m], 'FedOpt bucket')
            L.check(lib.fsagg_server_opt_step_f32(
                param[o:o + m].data_ptr(), avg[o:o + m].data_ptr(),
                st[0][o:o + m].data_ptr(),
                st[1][o:o + m].data_ptr() if st[1] is not None else None,
                m, ctypes.byref(hp), _stream(param.device)),
                'fsagg_server_opt_step_f32')
        st[2] += 1
        self._rounds += 1
        views = layout.unpack(param)
        with torch.no_grad():
            for k in step_keys:
                named[k].data.copy_(views[k])
        return self.model.state_dict()

    def _params(self, first, step):
        hp = L.OptParams()
        lr = self._lr()
        hp.lr = lr
        hp.weight_decay = self.weight_decay
        if self.opt_type == 'SGD':
            hp.kind = L.FSAGG_OPT_SGD
            hp.momentum = self.momentum
            hp.dampening = self.dampening
            hp.flags = (L.FSAGG_OPT_NESTEROV if self.nesterov else 0) | \
                (L.FSAGG_OPT_FIRST_STEP if first else 0)
        else:
            hp.kind = L.FSAGG_OPT_ADAM
            hp.beta1, hp.beta2, hp.eps = self.beta1, self.beta2, self.eps
            bc1 = 1 - self.beta1**step
            bc2 = 1 - self.beta2**step
            hp.step_size = lr / bc1
            hp.bias_correction2_sqrt = bc2**0.5
            hp.flags = L.FSAGG_OPT_FIRST_STEP if first else 0
        return hp


__all__ = ['FedOptAggregator']
