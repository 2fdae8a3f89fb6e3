"""Bulyan (federatedscope/core/aggregators/bulyan_aggregator.py:6-106):
multi-Krum selection of n - int(2·rate·f) clients (device distance matrix,
host score/sort as the reference), then a coordinate-wise trimmed mean over
the selected rows with k = int(rate·f), divided by gamma = |selected| - 2k,
plus init — all on the GPU over the one staged client stack."""
import torch

from ... import ops
from ._engine import _first_device
from .clients_avg_aggregator import ClientsAvgAggregator
from .krum_aggregator import krum_scores


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
        D = D.cpu()
        scores = krum_scores(D, self.byzantine_node_num)
        index_order = torch.sort(scores)[1].numpy()
        keep = n - int(2 * self.sample_client_rate * self.byzantine_node_num)
        sel = [int(i) for i in index_order[:max(keep, 0)]]
        self.last_selection = sel
        k = int(self.sample_client_rate * self.byzantine_node_num)
        gamma = len(sel) - 2 * k
        out = self._run_pieces(st.subset(sel), lambda rs, o, lo, hi:
                               ops.trimmed_mean_rows(rs, k, o, divisor=gamma,
                                                     base=base, lo=lo, hi=hi))
        return self._emit(layout, out, list(models[0][1].keys()), out_dev)
