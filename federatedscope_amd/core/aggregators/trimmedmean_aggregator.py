"""Coordinate-wise trimmed mean (federatedscope/core/aggregators/
trimmedmean_aggregator.py:10-57) on the GPU: drop the k = int(n·ratio)
largest and smallest of each coordinate, average the rest, add init — one
fsagg_trimmed_mean_rows_f32 launch over the clients' rows."""
from ... import ops
from ._engine import _first_device
from .clients_avg_aggregator import ClientsAvgAggregator


class TrimmedmeanAggregator(ClientsAvgAggregator):
    def __init__(self, model=None, device='cpu', config=None):
        super().__init__(model, device, config)
        self.excluded_ratio = \
            config.aggregator.BFT_args.trimmedmean_excluded_ratio
        self.byzantine_node_num = config.aggregator.byzantine_node_num
        assert 2 * self.byzantine_node_num + 2 < config.federate.client_num, \
            "it should be satisfied that 2*byzantine_node_num + 2 < client_num"
        assert self.excluded_ratio < 0.5

    def aggregate(self, agg_info):
        models = agg_info["client_feedback"]
        out_dev = _first_device(models[0][1])
        st = self._stage_all(models)
        layout = st.layout
        n = len(models)
        k = int(n * self.excluded_ratio)
        base = self._base(layout, self.model.state_dict(), as_float=True)
        out = self._run_pieces(st, lambda rs, o, lo, hi: ops.trimmed_mean_rows(
            rs, k, o, base=base, lo=lo, hi=hi))
        return self._emit(layout, out, list(models[0][1].keys()), out_dev)
