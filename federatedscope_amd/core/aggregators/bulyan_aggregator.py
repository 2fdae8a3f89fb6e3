"""Bulyan (federatedscope/core/aggregators/bulyan_aggregator.py:6-106):
multi-Krum selection of n - int(2·rate·f) clients (device distance matrix,
certified as in krum_aggregator; host score/sort as the reference), then a coordinate-wise trimmed mean over
the selected rows with k = int(rate·f), divided by gamma = |selected| - 2k,
plus init — all on the GPU over the one staged client stack."""
from ... import ops
from ._engine import _first_device
from .clients_avg_aggregator import ClientsAvgAggregator


class BulyanAggregator(ClientsAvgAggregator):
    def __init__(self, model=None, device='cpu', config=None):
        super().__init__(model, device, config)
        self.byzantine_node_num = config.aggregator.byzantine_node_num
        self.sample_client_rate = config.federate.sample_client_rate
        assert 4 * self.byzantine_node_num + 3 <= config.federate.client_num

    def aggregate(self, agg_info):
        models = agg_info["client_feedback"]
        out_dev = _first_device(models[0][1])
        st = self._stage_all(models)
        layout = st.layout
        n = len(models)
        D = self._pairdist(st)
        # the init model's table is built while the distance kernels run
        base = self._base(layout, self.model.state_dict(), as_float=True)
        keep = n - int(2 * self.sample_client_rate * self.byzantine_node_num)
        # the trimmed mean does not depend on the selected rows' order: the
        # Gram path's bounds need only certify the selected set
        _, _, index_order = self._certified_order(
            st, D.cpu(), self.byzantine_node_num, max(keep, 0), ordered=False)
        sel = [int(i) for i in index_order[:max(keep, 0)]]
        self.last_selection = sel
        k = int(self.sample_client_rate * self.byzantine_node_num)
        gamma = len(sel) - 2 * k
        out = self._run_pieces(st.subset(sel), lambda rs, o, lo, hi:
                               ops.trimmed_mean_rows(rs, k, o, divisor=gamma,
                                                     base=base, lo=lo, hi=hi))
        return self._emit(layout, out, list(models[0][1].keys()), out_dev)
