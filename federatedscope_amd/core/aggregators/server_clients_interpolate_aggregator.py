"""Server/clients interpolation (federatedscope/core/aggregators/
server_clients_interpolate_aggregator.py:4-30): FedAvg of the clients, then a
second weighted average of [(1-beta, global model), (beta, client average)]
— both passes on the GPU, the intermediate average never leaves HBM."""
from collections import OrderedDict

from ._engine import _first_device, fedavg_weights
from .clients_avg_aggregator import ClientsAvgAggregator


class ServerClientsInterpolateAggregator(ClientsAvgAggregator):
    def __init__(self, model=None, device='cpu', config=None, beta=1.0):
        super().__init__(model, device, config)
        self.beta = beta

    def aggregate(self, agg_info):
        models = agg_info["client_feedback"]
        elem_each_client = next(iter(models))
        assert len(elem_each_client) == 2, f"Require (sample_size, " \
                                           f"model_para) tuple for each " \
                                           f"client, i.e., len=2, but got " \
                                           f"len={len(elem_each_client)}"
        out_dev = _first_device(models[0][1])
        w1 = self._weights(models)
        lay1, flat1, extra1, keys1 = self._weighted_avg_device(models, w1)
        avg = lay1.unpack(flat1)          # device views, no copy
        avg.update(extra1)
        avg = OrderedDict((k, avg[k]) for k in keys1)
        glob = self.model.state_dict()
        pair = [((1 - self.beta), glob), (self.beta, avg)]
        w2 = fedavg_weights([s for s, _ in pair],
                            self.cfg.federate.ignore_weight)
        lay2, flat2, extra2, keys2 = self._weighted_avg_device(pair, w2)
        return self._emit(lay2, flat2, keys2, out_dev, extra2)
