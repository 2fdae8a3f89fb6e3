"""The server-side aggregation trigger around the device engine.

Reproduces the part of federatedscope/core/workers/server.py that feeds the
hot path:

* callback_funcs_model_para (server.py:929-988): buffer an upload under
  msg_buffer['train'][round][sender] (stale ones in staled_msg_buffer, too old
  ones dropped), optionally dequantise it (on the device, fused with the
  staging copy — core/compression/wire.py), feed online aggregation;
* check_and_move_on (:315-383, count-based part): aggregate once
  sample_client_num uploads of the current round are in;
* _perform_federated_aggregation (:437-490): msg_list in arrival order plus
  stale messages, the staleness list, agg_info, aggregate(),
  merge_param_dict + load_state_dict.

With ``stage_on_arrival`` every current-round upload is copied into its HBM
slot as it arrives (DeviceIngress), so the host→device traffic overlaps the
wait for the remaining clients instead of sitting inside aggregate().
"""
from collections import deque

from ..auxiliaries.utils import merge_param_dict
from .ingress import DeviceIngress


class AggregationServer:
    """``model`` / ``aggregator`` may be lists (the reference's
    ``model_num > 1``: a client uploads ``(sample_size, [para_0, …])`` and
    model i is aggregated by aggregator i, server.py:442-488).
    ``recover_fun`` is the server's secret-sharing recovery (passed in
    agg_info, server.py:481); ``monitor`` an object with the reference
    Monitor's ``calc_model_metric(global_state, msg_list, rnd)`` hook
    (server.py:473-475); ``keep_history`` how many rounds' results to keep
    in ``history`` (0: none — each result is a model-sized dict, on the GPU
    when the clients are)."""

    def __init__(self, model, aggregator, sample_client_num,
                 staleness_toleration=0, stage_on_arrival=True,
                 online_aggr=False, dequantize=False, device=None,
                 recover_fun=None, monitor=None, keep_history=0):
        self.models = list(model) if isinstance(model, (list, tuple)) \
            else [model]
        self.aggregators = list(aggregator) if isinstance(
            aggregator, (list, tuple)) else [aggregator]
        if len(self.models) != len(self.aggregators):
            raise ValueError('%d models for %d aggregators' %
                             (len(self.models), len(self.aggregators)))
        self.model_num = len(self.models)
        self.model = self.models[0]
        self.aggregator = self.aggregators[0]
        self.sample_client_num = sample_client_num
        self.staleness_toleration = staleness_toleration
        self.stage_on_arrival = stage_on_arrival and not online_aggr
        self.online_aggr = online_aggr
        self.dequantize = dequantize
        self.device = device
        self.recover_fun = recover_fun
        self.monitor = monitor
        self.state = 0
        self.msg_buffer = {'train': {}}
        self.staled_msg_buffer = []
        self.dropout_num = 0
        self.rejected_uploads = []
        self.ingresses = [None] * self.model_num
        self.history = deque(maxlen=keep_history) if keep_history else None
        if online_aggr:
            self.aggregator.reset()

    @property
    def ingress(self):
        return self.ingresses[0]

    # -- server.py:929-988 ---------------------------------------------------
    def _stage(self, idx, para, prev, sender=None):
        """Stage model ``idx``'s part of an upload on arrival (or keep it as
        it came when its layout differs from the round's)."""
        staged_quant = self.dequantize
        ing = self.ingresses[idx]
        if ing is None:
            ing = self.ingresses[idx] = DeviceIngress(
                para, self.sample_client_num, device=self.device,
                quantized=staged_quant)
        # a sender that uploads twice in one round overwrites its buffer
        # entry (server.py:966-970): reuse its stack row
        slot = prev.slot if getattr(prev, 'ingress', None) is ing else None
        if staged_quant:
            # dequantised on the device as the upload is staged
            return ing.receive_quantized(None, para, slot=slot)[1]
        if not ing.accepts(para):
            return para
        return ing.receive(None, para, slot=slot, tag=sender)[1]

    def callback_funcs_model_para(self, round, sender, content):
        staged_quant = self.dequantize and self.stage_on_arrival and \
            round == self.state
        if self.dequantize and not staged_quant:
            from ..compression import symmetric_uniform_dequantization
            sample_size, quant_model = content
            if isinstance(quant_model, list):       # multiple models
                quant_model = [symmetric_uniform_dequantization(x)
                               for x in quant_model]
            else:
                quant_model = symmetric_uniform_dequantization(quant_model)
            content = (sample_size, quant_model)
        if round == self.state:
            if self.stage_on_arrival:
                prev = self.msg_buffer['train'].get(round, {}).get(sender)
                size, para = content
                if self.model_num == 1:
                    para = self._stage(0, para, prev[1] if prev else None,
                                       sender)
                else:
                    para = [self._stage(i, p, prev[1][i] if prev else None,
                                        sender)
                            for i, p in enumerate(para)]
                content = (size, para)
            self.msg_buffer['train'].setdefault(round, dict())[sender] = \
                content
        elif round >= self.state - self.staleness_toleration:
            self.staled_msg_buffer.append((round, sender, content))
        else:
            self.dropout_num += 1
        if self.online_aggr:
            self.aggregator.inc(content)
        return self.check_and_move_on()

    # -- server.py:315-383 (count-based) ---------------------------------------
    def check_and_move_on(self):
        buf = self.msg_buffer['train'].get(self.state, {})
        if len(buf) < self.sample_client_num:
            return False
        if self._drop_rejected(buf) and len(buf) < self.sample_client_num:
            return False            # wait for uploads in their place
        self._perform_federated_aggregation()
        self.msg_buffer['train'].pop(self.state, None)
        self.state += 1
        self.staled_msg_buffer.clear()       # server.py:365
        for ing in self.ingresses:
            if ing is not None:
                ing.reset()
        if self.online_aggr:
            self.aggregator.reset()
        return True

    def _drop_rejected(self, buf):
        """Uploads whose base64 text the device decode rejected (a character
        outside the alphabet in the tensor data: DeviceIngress.rejected) are
        removed from this round's buffer by sender and recorded in
        ``rejected_uploads`` as (round, sender, reason) — the reference's
        receive path raises on such a message before it is ever buffered.
        Returns whether any was dropped."""
        dropped = False
        for ing in self.ingresses:
            if ing is None:
                continue
            for sender, reason in ing.rejected():
                if buf.pop(sender, None) is not None:
                    self.rejected_uploads.append((self.state, sender,
                                                  reason))
                    dropped = True
        return dropped

    # -- server.py:437-490 ----------------------------------------------------
    def _perform_federated_aggregation(self):
        train_msg_buffer = self.msg_buffer['train'][self.state]
        aggregated_num = 0
        results = []
        for model_idx in range(self.model_num):
            model = self.models[model_idx]
            aggregator = self.aggregators[model_idx]
            msg_list = []
            staleness = []
            for client_id in train_msg_buffer:
                size, para = train_msg_buffer[client_id]
                msg_list.append((size, para) if self.model_num == 1 else
                                (size, para[model_idx]))
                staleness.append((client_id, 0))
            for state, client_id, content in self.staled_msg_buffer:
                size, para = content
                msg_list.append((size, para) if self.model_num == 1 else
                                (size, para[model_idx]))
                staleness.append((client_id, self.state - state))
            if self.monitor is not None:
                self.monitor.calc_model_metric(self.models[0].state_dict(),
                                               msg_list, rnd=self.state)
            aggregated_num = len(msg_list)
            agg_info = {
                'client_feedback': msg_list,
                'recover_fun': self.recover_fun,
                'staleness': staleness,
            }
            result = aggregator.aggregate(agg_info)
            merged = merge_param_dict(model.state_dict().copy(), result)
            model.load_state_dict(merged, strict=False)
            results.append(result)
        if self.history is not None:
            self.history.append(results[0] if self.model_num == 1 else
                                results)
        return aggregated_num
