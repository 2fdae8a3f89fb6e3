"""FedOpt [Reddi et al., 2021] (federatedscope/core/aggregators/
fedopt_aggregator.py:7-44) with the server-optimizer step on the GPU.

aggregate(): FedAvg of the clients into a device bucket (bit-exact, as
ClientsAvgAggregator), then ONE fused pass fsagg_server_opt_step_f32 per
parameter that forms g = model − avg and applies the torch.optim step of the
configured optimizer — SGD (momentum, dampening, nesterov), Adam / AdamW
(amsgrad), Adagrad (lr_decay, initial accumulator) or RMSprop (momentum,
centered); weight decay and maximize for all — to the server model's
parameters and the per-parameter optimizer state, which stays resident in
HBM across rounds.  The updated parameters are written back into ``self.model`` and
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

# torch.optim optimizers the device step implements (optimizer_builder.py:
# 53-56 builds any torch.optim class by name; these are the ones with a
# single-tensor elementwise step)
_SUPPORTED = ('SGD', 'Adam', 'AdamW', 'Adagrad', 'RMSprop')
# keyword arguments that do not change the arithmetic of a single-tensor CPU
# step (the reference's optimizer runs on CPU tensors)
_IGNORED = ('foreach', 'fused', 'capturable', 'differentiable')


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
        for k in _IGNORED:
            opt.pop(k, None)
        # the constructor arguments as configured (the loop below consumes
        # ``opt``)
        self.opt_kwargs = dict(opt)
        self.maximize = bool(opt.pop('maximize', False))
        t = self.opt_type
        # torch.optim defaults per class
        self.weight_decay = float(opt.pop('weight_decay',
                                          1e-2 if t == 'AdamW' else 0.0))
        self.amsgrad = False
        if t == 'SGD':
            self.momentum = float(opt.pop('momentum', 0.0))
            self.dampening = float(opt.pop('dampening', 0.0))
            self.nesterov = bool(opt.pop('nesterov', False))
        elif t in ('Adam', 'AdamW'):
            betas = opt.pop('betas', (0.9, 0.999))
            self.beta1, self.beta2 = float(betas[0]), float(betas[1])
            self.eps = float(opt.pop('eps', 1e-8))
            self.amsgrad = bool(opt.pop('amsgrad', False))
            self.decoupled = t == 'AdamW' or bool(
                opt.pop('decoupled_weight_decay', False))
        elif t == 'Adagrad':
            self.lr_decay = float(opt.pop('lr_decay', 0.0))
            self.init_acc = float(opt.pop('initial_accumulator_value', 0.0))
            self.eps = float(opt.pop('eps', 1e-10))
        else:   # RMSprop
            self.alpha = float(opt.pop('alpha', 0.99))
            self.eps = float(opt.pop('eps', 1e-8))
            self.momentum = float(opt.pop('momentum', 0.0))
            self.centered = bool(opt.pop('centered', False))
        if opt:
            raise TypeError('%s got unexpected arguments %s' %
                            (self.opt_type, sorted(opt)))
        self._validate()
        fo = config.fedopt
        self._annealing = bool(getattr(fo, 'annealing', False))
        self._anneal_step = int(getattr(fo, 'annealing_step_size', 2000))
        self._anneal_gamma = float(getattr(fo, 'annealing_gamma', 0.5))
        self._rounds = 0
        # optimizer state per parameter name, as torch.optim keeps it:
        # name -> [state0, state1, state2, steps]
        self._state = {}

    def _validate(self):
        """The argument checks of the torch.optim constructors the
        reference's get_optimizer calls (optimizer_builder.py:53-56), with
        their messages: an invalid config fails here as it does there."""
        t = self.opt_type

        def need(ok, msg, v):
            if not ok:
                raise ValueError(msg % (v, ))
        need(0.0 <= self.lr0, 'Invalid learning rate: %s', self.lr0)
        if t in ('Adam', 'AdamW', 'Adagrad', 'RMSprop'):
            need(0.0 <= self.eps, 'Invalid epsilon value: %s', self.eps)
        if t == 'SGD':
            need(0.0 <= self.momentum, 'Invalid momentum value: %s',
                 self.momentum)
        if t in ('Adam', 'AdamW'):
            need(0.0 <= self.beta1 < 1.0,
                 'Invalid beta parameter at index 0: %s', self.beta1)
            need(0.0 <= self.beta2 < 1.0,
                 'Invalid beta parameter at index 1: %s', self.beta2)
        need(0.0 <= self.weight_decay, 'Invalid weight_decay value: %s',
             self.weight_decay)
        if t == 'SGD' and self.nesterov and (self.momentum <= 0 or
                                             self.dampening != 0):
            raise ValueError('Nesterov momentum requires a momentum and zero '
                             'dampening')
        if t == 'Adagrad':
            need(0.0 <= self.lr_decay, 'Invalid lr_decay value: %s',
                 self.lr_decay)
            need(0.0 <= self.init_acc,
                 'Invalid initial_accumulator_value value: %s', self.init_acc)
        if t == 'RMSprop':
            need(0.0 <= self.momentum, 'Invalid momentum value: %s',
                 self.momentum)
            need(0.0 <= self.alpha, 'Invalid alpha value: %s', self.alpha)

    def _lr(self):
        if not self._annealing:
            return self.lr0
        return self.lr0 * self._anneal_gamma ** (self._rounds //
                                                 self._anneal_step)

    def _new_model(self, agg_info):
        """super().aggregate(agg_info) of the reference (:30): the FedAvg —
        or, with federate.use_ss, the secret-sharing average — as (layout,
        fp32 bucket, {other-dtype key: device tensor})."""
        models = agg_info["client_feedback"]
        if self.cfg.federate.use_ss:
            recover_fun = agg_info.get('recover_fun')
            avg = self._ss_avg(models, recover_fun)
            dev = self.compute_device
            avg = OrderedDict((k, torch.as_tensor(v)) for k, v in avg.items())
            layout = self._layout(avg)
            extra = OrderedDict((k, avg[k].to(dev)) for k in layout.other)
            return layout, self._bucket(layout, avg), extra
        weights = fedavg_weights([s for s, _ in models],
                                 self.cfg.federate.ignore_weight)
        layout, avg, extra, _ = self._weighted_avg_device(models, weights)
        return layout, avg, extra

    def _states(self, key, like):
        """The optimizer state of parameter ``key`` (created on its first
        step, shaped like ``like``: flat, on the compute device)."""
        st = self._state.get(key)
        if st is None:
            t = self.opt_type
            z = lambda: torch.zeros_like(like)  # noqa: E731
            if t == 'SGD':
                st = [z() if self.momentum != 0.0 else None, None, None]
            elif t in ('Adam', 'AdamW'):
                st = [z(), z(), z() if self.amsgrad else None]
            elif t == 'Adagrad':
                st = [torch.full_like(like, self.init_acc), None, None]
            else:
                st = [z(), z() if self.momentum > 0 else None,
                      z() if self.centered else None]
            st.append(0)
            self._state[key] = st
        return st

    def _step(self, fn, param, avg, st):
        """One optimizer step of a contiguous device parameter range."""
        hp = self._params(first=(st[3] == 0), step=st[3] + 1)
        L.check(fn(param.data_ptr(), avg.data_ptr(),
                   *[t.data_ptr() if t is not None else None
                     for t in st[:3]],
                   param.numel(), ctypes.byref(hp), _stream(param.device)),
                'fedopt step')
        st[3] += 1

    def aggregate(self, agg_info):
        layout, avg, extra = self._new_model(agg_info)
        lib = L.load()
        named = OrderedDict(self.model.named_parameters())
        # parameters the aggregate holds (fedopt_aggregator.py:37-40); other
        # state_dict entries (buffers) are returned unchanged
        step_keys = [k for k in named if k in layout.keys]
        for k in named:
            if k in extra and extra[k].dtype != torch.float64:
                raise NotImplementedError(
                    'FedOpt on %s parameter %r' % (extra[k].dtype, k))
        dev = self.compute_device
        inplace = bool(step_keys) and all(
            named[k].device == dev and named[k].dtype == torch.float32 and
            named[k].is_contiguous() and named[k].data_ptr() % 16 == 0
            for k in step_keys)
        if inplace:
            # parameters already on the compute device: the optimizer steps
            # them in place (as torch.optim's step does), no bucket copy of
            # the model in or out
            for k in step_keys:
                o, m = layout.offsets[k], layout.numels[k]
                _check_f32_cuda(avg[o:o + m], 'FedOpt bucket')
                self._step(lib.fsagg_server_opt_step_f32,
                           named[k].data.view(-1), avg[o:o + m],
                           self._states(k, avg[o:o + m]))
        elif step_keys:
            param = self._bucket(layout, OrderedDict(
                (k, named[k].detach() if k in named else torch.zeros(
                    layout.shapes[k])) for k in layout.keys))
            for k in step_keys:      # per key: params the optimizer owns
                o, m = layout.offsets[k], layout.numels[k]
                for t in (param, avg):
                    _check_f32_cuda(t[o:o + m], 'FedOpt bucket')
                self._step(lib.fsagg_server_opt_step_f32, param[o:o + m],
                           avg[o:o + m], self._states(k, avg[o:o + m]))
            views = layout.unpack(param)
            with torch.no_grad():
                for k in step_keys:
                    named[k].data.copy_(views[k])
        for k in named:              # float64 parameters, one key each
            if k not in extra:
                continue
            p64 = named[k].detach().to(dev, torch.float64).contiguous()
            a64 = extra[k].to(dev, torch.float64).contiguous()
            self._step(lib.fsagg_server_opt_step_f64, p64, a64,
                       self._states(k, p64.view(-1)))
            with torch.no_grad():
                named[k].data.copy_(p64)
        self._rounds += 1
        return self.model.state_dict()

    def _params(self, first, step):
        hp = L.OptParams()
        lr = self._lr()
        t = self.opt_type
        hp.lr = lr
        hp.weight_decay = self.weight_decay
        flags = (L.FSAGG_OPT_FIRST_STEP if first else 0) | \
            (L.FSAGG_OPT_MAXIMIZE if self.maximize else 0)
        if t == 'SGD':
            hp.kind = L.FSAGG_OPT_SGD
            hp.momentum = self.momentum
            hp.dampening = self.dampening
            flags |= L.FSAGG_OPT_NESTEROV if self.nesterov else 0
        elif t in ('Adam', 'AdamW'):
            hp.kind = L.FSAGG_OPT_ADAM
            hp.beta1, hp.beta2, hp.eps = self.beta1, self.beta2, self.eps
            bc1 = 1 - self.beta1**step
            bc2 = 1 - self.beta2**step
            hp.step_size = lr / bc1
            hp.bias_correction2_sqrt = bc2**0.5
            hp.decay_mul = 1 - lr * self.weight_decay
            flags |= (L.FSAGG_OPT_AMSGRAD if self.amsgrad else 0) | \
                (L.FSAGG_OPT_DECOUPLED if self.decoupled else 0)
        elif t == 'Adagrad':
            hp.kind = L.FSAGG_OPT_ADAGRAD
            hp.eps = self.eps
            hp.clr = lr / (1 + (step - 1) * self.lr_decay)
        else:
            hp.kind = L.FSAGG_OPT_RMSPROP
            hp.alpha, hp.eps, hp.momentum = self.alpha, self.eps, \
                self.momentum
            flags |= L.FSAGG_OPT_CENTERED if self.centered else 0
        hp.flags = flags
        return hp


__all__ = ['FedOptAggregator']
