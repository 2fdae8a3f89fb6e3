"""Coordinate-wise median (federatedscope/core/aggregators/
median_aggregator.py:10-52) on the GPU: fsagg_coord_median_rows_f32 computes
(median(T) - median(-T))/2 per coordinate (bit-exact) and adds the server's
init model in the same kernel."""
from ... import ops
from ._engine import _first_device
from .clients_avg_aggregator import ClientsAvgAggregator


class MedianAggregator(ClientsAvgAggregator):
    def __init__(self, model=None, device='cpu', config=None):
        super().__init__(model, device, config)
        self.byzantine_node_num = config.aggregator.byzantine_node_num
        assert 2 * self.byzantine_node_num + 2 < config.federate.client_num, \
            "it should be satisfied that 2*byzantine_node_num + 2 < client_num"

    def aggregate(self, agg_info):
        models = agg_info["client_feedback"]
        out_dev = _first_device(models[0][1])
        st = self._stage_all(models)
        layout = st.layout
        base = self._base(layout, self.model.state_dict(), as_float=True)
        out = self._run_pieces(st, lambda rs, o, lo, hi: ops.coord_median_rows(
            rs, o, base=base, lo=lo, hi=hi))
        return self._emit(layout, out, list(models[0][1].keys()), out_dev)
