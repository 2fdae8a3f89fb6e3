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
from ..auxiliaries.utils import merge_param_dict
from .ingress import DeviceIngress


class AggregationServer:
    def __init__(self, model, aggregator, sample_client_num,
                 staleness_toleration=0, stage_on_arrival=True,
                 online_aggr=False, dequantize=False, device=None):
        self.model = model
        self.aggregator = aggregator
        self.sample_client_num = sample_client_num
        self.staleness_toleration = staleness_toleration
        self.stage_on_arrival = stage_on_arrival and not online_aggr
        self.online_aggr = online_aggr
        self.dequantize = dequantize
        self.device = device
        self.state = 0
        self.msg_buffer = {'train': {}}
        self.staled_msg_buffer = []
        self.dropout_num = 0
        self.ingress = None
        self.history = []
        if online_aggr:
            self.aggregator.reset()

    # -- server.py:929-988 ---------------------------------------------------
    def callback_funcs_model_para(self, round, sender, content):
        staged_quant = self.dequantize and self.stage_on_arrival and \
            round == self.state
        if self.dequantize and not staged_quant:
            from ..compression import symmetric_uniform_dequantization
            sample_size, quant_model = content
            content = (sample_size,
                       symmetric_uniform_dequantization(quant_model))
        if round == self.state:
            if self.stage_on_arrival:
                if self.ingress is None:
                    self.ingress = DeviceIngress(content[1],
                                                 self.sample_client_num,
                                                 device=self.device,
                                                 quantized=staged_quant)
                # a sender that uploads twice in one round overwrites its
                # buffer entry (server.py:966-970): reuse its stack row
                prev = self.msg_buffer['train'].get(round, {}).get(sender)
                slot = prev[1].slot if prev and getattr(
                    prev[1], 'ingress', None) is self.ingress else None
                if staged_quant:
                    # dequantised on the device as the upload is staged
                    content = self.ingress.receive_quantized(*content,
                                                             slot=slot)
                else:
                    content = self.ingress.receive(*content, slot=slot)
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
        self._perform_federated_aggregation()
        self.msg_buffer['train'].pop(self.state, None)
        self.state += 1
        self.staled_msg_buffer.clear()       # server.py:365
        if self.ingress is not None:
            self.ingress.reset()
        if self.online_aggr:
            self.aggregator.reset()
        return True

    # -- server.py:437-490 ----------------------------------------------------
    def _perform_federated_aggregation(self):
        train_msg_buffer = self.msg_buffer['train'][self.state]
        msg_list = []
        staleness = []
        for client_id in train_msg_buffer:
            msg_list.append(train_msg_buffer[client_id])
            staleness.append((client_id, 0))
        for state, client_id, content in self.staled_msg_buffer:
            msg_list.append(content)
            staleness.append((client_id, self.state - state))
        agg_info = {
            'client_feedback': msg_list,
            'recover_fun': None,
            'staleness': staleness,
        }
        result = self.aggregator.aggregate(agg_info)
        merged = merge_param_dict(self.model.state_dict().copy(), result)
        self.model.load_state_dict(merged, strict=False)
        self.history.append(result)
        return result
