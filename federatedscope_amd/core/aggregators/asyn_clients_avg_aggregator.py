"""Staleness-discounted FedAvg (federatedscope/core/aggregators/
asyn_clients_avg_aggregator.py:6-84), on the GPU.

Weights: (size_i/total or 1/n) · 1/(1+τ_i)^factor in double (:42-51,:67-73);
every key is cast to float (:74-77); the result is init + avg, fused into the
weighted-sum kernel's epilogue (fl32(init + acc))."""
from ._engine import _first_device
from .clients_avg_aggregator import ClientsAvgAggregator


class AsynClientsAvgAggregator(ClientsAvgAggregator):
    def __init__(self, model=None, device='cpu', config=None):
        super().__init__(model, device, config)

    def aggregate(self, agg_info):
        models = agg_info["client_feedback"]
        # use_ss: the reference hands recover_fun to _para_weighted_avg but
        # never applies it on this path (:25-31, :53-84); neither do we
        staleness = [x[1] for x in agg_info['staleness']]
        weights = self._asyn_weights(models, staleness)
        out_dev = _first_device(models[0][1])
        layout, flat, extra, keys = self._weighted_avg_device(
            models, weights, as_float=True,
            base_model=self.model.state_dict())
        return self._emit(layout, flat, keys, out_dev, extra)

    def discount_func(self, staleness):
        return (1.0 /
                ((1.0 + staleness)**self.cfg.asyn.staleness_discount_factor))

    def _asyn_weights(self, models, staleness):
        total = 0
        for s, _ in models:
            total += s
        out = []
        for i, (s, _) in enumerate(models):
            w = 1.0 / len(models) if self.cfg.federate.ignore_weight \
                else s / total
            w *= self.discount_func(staleness[i])
            out.append(w)
        return out
