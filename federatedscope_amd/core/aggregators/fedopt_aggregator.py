"""FedOpt (federatedscope/core/aggregators/fedopt_aggregator.py:7-44).

The server-optimizer epilogue is SURVEY §8(f) rank 2 ("next"): it is not on
the device path yet, and this drop-in says so instead of computing on the
host."""
from .clients_avg_aggregator import ClientsAvgAggregator


class FedOptAggregator(ClientsAvgAggregator):
    def __init__(self, config, model, device='cpu'):
        super().__init__(model, device, config)
        raise NotImplementedError(
            'FedOptAggregator: the fused server-optimizer step is not '
            'implemented on the device path yet')
